"""Kokoro end to end (duration graph + main graph + generator) on the CPU oracle, checked stage by
stage against an independent float PyTorch restatement of Kokoro's front half
(tests/kokoro_front_ref.py) and generator (tests/kokoro_ref.py).

The oracle rounds conv inputs / kernels to f16 (ggml conv_1d's im2col) and evaluates GELU through
ggml's f16 table, where PyTorch stays in fp32: the bar is the f16 level, every named intermediate
within 5e-3 of its scale.  The generator stage is fed the runner's own decoder output and F0 (a
Hz-scale F0 difference at the f16 level shifts the sine phases that the PCM then carries), as
tests/test_kokoro_cpu.py checks it."""
import numpy as np
import pytest

import kokoro_front_ref
import kokoro_ref
import py_oracle
import ttship

TINY = dict(gen=dict(in_channels=32, style_dim=16), hidden=64, n_heads=4, ffn=128, embd=32, d_model=32, dec_dim=64, asr_res_dim=8,
            max_tokens=16, max_total=96, n_recurrence=3, n_voice_rows=20)


def tokens(n, seed, vocab=178):
    rng = np.random.default_rng(seed)
    t = rng.integers(1, vocab, n).astype(np.int32)
    t[0] = t[-1] = 0  # the pad / boundary id the phonemizer wraps a prompt in
    return t


def close(got, ref, name, rel=5e-3):
    ref = ref.detach().contiguous().numpy().reshape(-1) if hasattr(ref, "detach") else np.asarray(ref).reshape(-1)
    got = None if got is None else np.asarray(got).reshape(-1)
    assert got is not None and got.shape == ref.shape, (name, None if got is None else got.shape, ref.shape)
    scale = float(np.max(np.abs(ref)))
    err = float(np.max(np.abs(got - ref)))
    assert err <= rel * max(scale, 1.0), f"{name}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("n,seed,wtype", [(7, 0, ttship.F32), (12, 1, ttship.F32), (9, 2, ttship.F16)])
def test_kokoro_model_oracle_matches_torch(n, seed, wtype):
    """wtype F16: the F16 GGUF (quantize -qt F16 -nqf): the torch restatement runs on the widened f16
    weights; the oracle's F16 mul_mats / convs also round their inputs to f16, inside the same bar."""
    cfg = ttship.kokoro_config(**TINY, debug_no_reuse=1, arena_bytes=1 << 30, weight_type=wtype)
    k = ttship.Kokoro(py_oracle.iface(8), cfg)
    try:
        W = k.weights()
        toks = tokens(n, seed)
        hidden, lens = k.durations(toks)
        taps = {}
        h_ref, probs, l_ref = kokoro_front_ref.durations(cfg, W, toks, taps)
        for name in ("albert_out", "duration_hidden_states", "duration_probs"):
            close(k.node(name, 0), taps[name], name)
        close(hidden, h_ref, "hidden")
        # lengths: identical wherever the torch sum is not within 1e-3 of a rounding boundary
        sums = probs.sum(-1).numpy()
        safe = np.abs(sums - np.floor(sums) - 0.5) > 1e-3
        assert np.array_equal(lens[safe], l_ref.numpy()[safe]), (lens, l_ref)
        assert lens.min() >= 1 and lens.max() <= cfg.max_dur and len(np.unique(lens)) > 1

        rng = np.random.default_rng(seed + 100)
        total = int(lens.sum())
        rand = rng.random((cfg.gen.harmonic_num + 1, 600 * total), dtype=np.float32)
        pcm = k.decode(toks, hidden, lens, rand)
        assert pcm.shape == (600 * total,) and np.all(np.isfinite(pcm))
        dtaps = {}
        kokoro_front_ref.decoder(cfg, W, toks, hidden, lens, dtaps)
        for name, v in dtaps.items():
            close(k.node(name), v, name)
        # generator stage from the runner's own features / F0 (tests/test_kokoro_cpu.py's bar)
        x = k.node("decoder_out").reshape(2 * total, cfg.gen.in_channels)
        f0 = k.node("f0_out")
        s2, _ = kokoro_front_ref.styles(W, n)
        ref = kokoro_ref.generator(cfg.gen, W, x, f0, s2.numpy(), rand, har_branch=k.node("har_spec"), f16=wtype == ttship.F16)
        err = float(np.max(np.abs(pcm[:-cfg.gen.hop] - ref[:-cfg.gen.hop])))
        assert err <= 2e-3 * float(np.max(np.abs(ref))), err
        assert float(np.std(pcm)) > 1e-2
    finally:
        k.close()


def test_kokoro_model_run_matches_stages_and_is_deterministic():
    cfg = ttship.kokoro_config(**TINY)
    k = ttship.Kokoro(py_oracle.iface(8), cfg)
    try:
        toks = tokens(9, 3)
        a = k.run(toks)
        b = k.run(toks)
        assert np.array_equal(a, b)
        hidden, lens = k.durations(toks)
        assert a.shape == (600 * int(lens.sum()),)
        c = k.decode(toks, hidden, lens)  # the runner's own seeded draws, as run() uses
        assert np.array_equal(a, c)
        assert k.last_graph_nodes(0) > 100 and k.last_graph_nodes(1) > k.last_graph_nodes(0)
    finally:
        k.close()


def test_kokoro_model_rejects_bad_inputs():
    cfg = ttship.kokoro_config(**TINY)
    k = ttship.Kokoro(py_oracle.iface(2), cfg)
    try:
        with pytest.raises(RuntimeError):
            k.durations(tokens(2, 0))  # fewer than 3 tokens: no voice row n - 3
        with pytest.raises(RuntimeError):
            k.durations(tokens(cfg.max_tokens + 1, 0))
        bad = tokens(5, 0)
        bad[2] = cfg.n_vocab
        with pytest.raises(RuntimeError):
            k.durations(bad)
        hidden, lens = k.durations(tokens(5, 0))
        with pytest.raises(RuntimeError):
            k.decode(tokens(5, 0), hidden, np.full(5, cfg.max_total, np.float32))  # beyond max_dur / max_total
    finally:
        k.close()
    with pytest.raises(RuntimeError):
        ttship.Kokoro(py_oracle.iface(1), ttship.kokoro_config(**dict(TINY, n_heads=5)))  # hidden % heads


def test_kokoro_model_fusion_coverage():
    """The HIP planner's view (no device): every LSTM recurrence fuses into per-step kernels, every
    AdaIN and conv chain of the decoder collapses."""
    cfg = ttship.kokoro_config(**TINY)
    k = ttship.Kokoro(py_oracle.iface(4), cfg)
    try:
        k.run(tokens(8, 5))
        d, nd = k.plan_stats(0), k.last_graph_nodes(0)
        m, nm = k.plan_stats(1), k.last_graph_nodes(1)
    finally:
        k.close()
    # 4 bidirectional recurrences over 8 tokens, each direction pair advanced by one launch per step:
    # a projection stash, 8 paired steps and one output write per pair
    assert d["lstm"] == 4 * (1 + 8 + 1), d
    assert m["lstm"] > 2 * 2 * 8 and m["adain"] > 0 and m["conv"] > 0, m
    assert d["unfused"] < nd // 8 and m["unfused"] < nm // 8, (d, m)


def test_kokoro_model_f16_weights_follow_quantize_rule():
    """weight_type F16 stores exactly the tensors kokoro_is_f16_compatible names (matrices and conv
    kernels; biases, norms, gamma / beta / alpha, embeddings and the voice pack stay F32), rounded to
    f16; durations stay close to the F32 model's."""
    cfg32 = ttship.kokoro_config(**TINY)
    cfg16 = ttship.kokoro_config(**TINY, weight_type=ttship.F16)
    a = ttship.Kokoro(py_oracle.iface(8), cfg32)
    b = ttship.Kokoro(py_oracle.iface(8), cfg16)
    try:
        w32, w16 = a.weights(), b.weights()
        assert w32.keys() == w16.keys()
        n16 = 0
        for name, v in w32.items():
            excluded = (any(x in name for x in ("voice_tensors", "bias", "gamma", "beta", "alpha")) or name.endswith(("embd", "norm"))
                        or name in ("stft_window", "harmonic_sampling_norm", "sampling_factor_scalar", "n_kernels_tensor", "one",
                                    "sqrt_tensor"))
            if np.array_equal(w16[name], v) and (excluded or v.size == v.shape[-1] and "kernel" not in name):
                continue  # F32 (excluded by the rule, or a 1-D tensor)
            assert not excluded, name
            n16 += 1
            assert np.array_equal(w16[name], v.astype(np.float16).astype(np.float32)), name
        assert n16 > 50
        toks = tokens(8, 4)
        h32, l32 = a.durations(toks)
        h16, l16 = b.durations(toks)
        assert np.max(np.abs(h16 - h32)) < 5e-2 * max(1.0, float(np.max(np.abs(h32))))
        p16 = b.decode(toks, h32, l32)
        p32 = a.decode(toks, h32, l32)
        assert p16.shape == p32.shape and np.all(np.isfinite(p16))
        # (the iSTFT head's phases amplify the f16 weight rounding: the two models' PCM are different
        # signals of the same scale, not an f16-level perturbation of each other)
        assert not np.array_equal(p16, p32) and 0.5 < float(np.std(p16)) / float(np.std(p32)) < 2.0
    finally:
        a.close()
        b.close()
