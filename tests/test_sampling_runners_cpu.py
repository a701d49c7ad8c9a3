"""Seeded sampling inside the runners, on the CPU oracle backend (host sampling path): each
runner's generate() with tts_sampling set equals a Python loop that decodes step by step and draws
with oracle/py_sampler.py (prompt b = stream b, call = step), with the runner's next-token rule
restated (Parler: next_decoder_token_ids, src/models/parler/model.cpp:778-785; Dia / Orpheus: the
sample itself).  The GPU side of the same bar is tests/test_sampling_runners_gpu.py."""
import numpy as np

import py_oracle
import py_sampler
import ttship

PARLER_TINY = dict(n_layers=2, hidden_size=128, n_attn_heads=4, ffn_size=256, output_vocab=1088, max_ctx=64,
                   prompt_vocab=512, max_positions=96)


def _py_sampler(cfg, NH, V):
    return py_sampler.Sampler(NH, V, temperature=cfg.temperature, top_k=cfg.top_k, top_p=cfg.top_p,
                              repetition_penalty=cfg.repetition_penalty, do_sample=bool(cfg.do_sample), seed=cfg.seed)


def test_parler_sampled_tokens_match_python_loop():
    B, steps = 2, 12
    pc = ttship.parler_config(batch=B, **PARLER_TINY)
    scfg = ttship.sampling(seed=2024, top_k=20, temperature=0.9, repetition_penalty=1.3)
    a = ttship.Parler(py_oracle.iface(4), pc)
    b = ttship.Parler(py_oracle.iface(4), pc)
    try:
        prompt = (np.arange(5 * B, dtype=np.int32).reshape(B, 5) * 53) % 512
        a.prefill(prompt)
        b.prefill(prompt)
        a.set_sampling(scfg)
        got = a.generate(steps)
        NH, V, bos, eos = pc.n_output_heads, pc.output_vocab, pc.bos_token, pc.eos_token
        samplers = [_py_sampler(scfg, NH, V) for _ in range(B)]
        hist = np.zeros((B, steps, NH), np.int32)
        seen = np.zeros((B, NH), bool)
        for s in range(steps):
            toks = np.full((B, NH), bos, np.int32)
            for h in range(NH):
                if s > h:
                    toks[:, h] = np.where(seen[:, h], eos, hist[:, s - 1, h])
            lg = b.decode(toks)
            for p in range(B):
                hist[p, s] = samplers[p].sample(lg[p], stream=p, call=s)
            seen |= hist[:, s] == eos
        assert np.array_equal(got, hist), f"{got}\n{hist}"
        assert len(np.unique(got)) > NH  # sampled, not greedy
    finally:
        a.close()
        b.close()


def test_greedy_remains_default_and_do_sample_zero_is_greedy():
    pc = ttship.parler_config(batch=1, **PARLER_TINY)
    a = ttship.Parler(py_oracle.iface(4), pc)
    b = ttship.Parler(py_oracle.iface(4), pc)
    try:
        prompt = np.array([[3, 9, 27, 81]], np.int32)
        a.prefill(prompt)
        b.prefill(prompt)
        b.set_sampling(ttship.sampling(do_sample=0))
        assert np.array_equal(a.generate(6), b.generate(6))
    finally:
        a.close()
        b.close()
