"""Seeded sampling end to end (north_star: "bit-exact sampled token IDs at fixed seed"): each runner's
generate() with tts_sampling set, HIP backend (device sampler inside the device-resident step loop)
vs the CPU oracle backend (host sampler, pinned to oracle/py_sampler.py by the CPU tests)."""
import numpy as np
import pytest

import py_oracle
import ttship

PARLER_TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=128,
                   prompt_vocab=512, max_positions=160)
DIA_TINY = dict(n_encoder_layers=1, n_decoder_layers=2, encoder_hidden_size=64, decoder_hidden_size=128, encoder_attn_heads=4,
                decoder_attn_heads=4, decoder_query_heads=2, head_size=32, encoder_ffn_size=128, decoder_ffn_size=256,
                max_generation_size=64, max_encoder_context_length=32)
ORPHEUS_WIDE = dict(n_layers=2, max_ctx=40)  # real widths and the 156 940-token vocabulary


@pytest.mark.gpu
@pytest.mark.parametrize("kw,batch,scfg", [
    (PARLER_TINY, 3, dict()),
    (PARLER_TINY, 2, dict(top_k=0, top_p=0.9, temperature=0.8, repetition_penalty=1.2)),
    ({}, 2, dict(top_k=50)),  # Parler-mini Q4_K at full depth and width
])
def test_parler_sampled_tokens(hip, kw, batch, scfg):
    cfg = ttship.parler_config(batch=batch, **kw)
    g = ttship.Parler(hip.iface(), cfg)
    c = ttship.Parler(py_oracle.iface(16), ttship.parler_config(batch=batch, **kw))
    try:
        prompt = (np.arange(6 * batch, dtype=np.int32).reshape(batch, 6) * 37 + 5) % cfg.prompt_vocab
        g.prefill(prompt)
        c.prefill(prompt)
        s = ttship.sampling(seed=31337, **scfg)
        g.set_sampling(s)
        c.set_sampling(s)
        steps = 6 if not kw else 14
        tg, tc = g.generate(steps), c.generate(steps)
        assert np.array_equal(tg, tc), f"{tg}\n{tc}"
        tg2, tc2 = g.generate(3), c.generate(3)  # the state (calls, penalties) carries over
        assert np.array_equal(tg2, tc2)
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_dia_sampled_tokens(hip):
    g = ttship.Dia(hip.iface(), ttship.dia_config(**DIA_TINY))
    c = ttship.Dia(py_oracle.iface(16), ttship.dia_config(**DIA_TINY))
    try:
        text = np.frombuffer(b"\x01 It's easy to tell the depth.", dtype=np.uint8).astype(np.int32)[:32]
        first = c.prefill(text, np.full(9, 1026, dtype=np.int32)).argmax(axis=1).astype(np.int32)
        g.prefill(text, np.full(9, 1026, dtype=np.int32))
        s = ttship.sampling(seed=4242, top_k=30, temperature=1.1)
        g.set_sampling(s)
        c.set_sampling(s)
        tg, tc = g.generate(first, 12), c.generate(first, 12)
        assert np.array_equal(tg, tc), f"{tg}\n{tc}"
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_orpheus_sampled_tokens_wide_vocab(hip):
    B = 2
    g = ttship.Orpheus(hip.iface(), ttship.orpheus_config(batch=B, **ORPHEUS_WIDE))
    c = ttship.Orpheus(py_oracle.iface(16), ttship.orpheus_config(batch=B, **ORPHEUS_WIDE))
    try:
        V = c.cfg.vocab_size
        prompt = (np.arange(6 * B, dtype=np.int32).reshape(B, 6) * 7919 + 3) % V
        first = c.prefill(prompt).argmax(axis=1).astype(np.int32)
        g.prefill(prompt)
        s = ttship.sampling(seed=99, top_k=50, repetition_penalty=1.1)
        g.set_sampling(s)
        c.set_sampling(s)
        tg, tc = g.generate(first, 8), c.generate(first, 8)
        assert np.array_equal(tg, tc), f"{tg}\n{tc}"
    finally:
        g.close()
        c.close()
