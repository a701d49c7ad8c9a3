"""Kokoro iSTFTNet generator runner on the CPU oracle (no GPU), checked against an independent
float32 PyTorch restatement of Kokoro's published generator (tests/kokoro_ref.py).

The oracle rounds conv inputs and kernels to f16 (ggml conv_1d's im2col) where PyTorch stays in
fp32, so the bar is the f16 level: every named intermediate within 2e-3 of its scale, PCM within
2e-3 of its peak.  The last `hop` samples are excluded: compute_window_squared_sum (util.cpp:203-217)
adds one frame past the end that torch.istft's envelope does not have (a reference quirk the
runner keeps)."""
import numpy as np
import pytest

import kokoro_ref
import py_oracle
import ttship

TINY = dict(in_channels=32, style_dim=16, max_frames=16)


def inputs(cfg, T, seed, f0=None):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((T, cfg.in_channels)) * 0.5).astype(np.float32)
    if f0 is None:
        f0 = rng.uniform(60, 300, T).astype(np.float32)
        f0[::3] = 0.0  # unvoiced frames (below voice_threshold)
    style = rng.standard_normal(cfg.style_dim).astype(np.float32)
    rand = rng.random((cfg.harmonic_num + 1, 300 * T), dtype=np.float32)
    return x, np.asarray(f0, np.float32), style, rand


@pytest.mark.parametrize("T,seed", [(4, 0), (7, 1)])
def test_kokoro_generator_oracle_matches_torch(T, seed):
    cfg = ttship.kokoro_gen_config(**TINY, debug_no_reuse=1, arena_bytes=256 << 20)
    k = ttship.KokoroGenerator(py_oracle.iface(8), cfg)
    try:
        x, f0, style, rand = inputs(cfg, T, seed)
        pcm = k.run(x, f0, style, rand)
        taps = {}
        ref = kokoro_ref.generator(cfg, k.weights(), x, f0, style, rand, taps, har_branch=k.node("har_spec"))
        for name, v in taps.items():
            got = k.node(name)
            v = v.contiguous().numpy().reshape(-1)
            assert got is not None and got.shape == v.shape, name
            scale = float(np.max(np.abs(v)))
            assert float(np.max(np.abs(got - v))) <= 2e-3 * max(scale, 1.0), name
        assert pcm.shape == (300 * T,) and np.all(np.isfinite(pcm))
        err = float(np.max(np.abs(pcm[:-cfg.hop] - ref[:-cfg.hop])))
        assert err <= 2e-3 * float(np.max(np.abs(ref))), err
        assert float(np.std(pcm)) > 1e-2  # not silent
        assert k.last_graph_nodes() > 500
    finally:
        k.close()


def test_kokoro_generator_deterministic_and_rand_default():
    cfg = ttship.kokoro_gen_config(**TINY)
    k = ttship.KokoroGenerator(py_oracle.iface(4), cfg)
    try:
        x, f0, style, rand = inputs(cfg, 3, 5)
        a, b = k.run(x, f0, style, rand), k.run(x, f0, style, rand)
        assert np.array_equal(a, b)
        c, d = k.run(x, f0, style), k.run(x, f0, style)  # runner's own seeded draws
        assert np.array_equal(c, d) and c.shape == a.shape
        assert k.samples_per_frame == 300
    finally:
        k.close()


def test_kokoro_generator_rejects_bad_config():
    cfg = ttship.kokoro_gen_config(**TINY, up_rates=[10, 5])  # 10*5*5 != 300
    with pytest.raises(RuntimeError):
        ttship.KokoroGenerator(py_oracle.iface(1), cfg)
    cfg = ttship.kokoro_gen_config(**TINY)
    k = ttship.KokoroGenerator(py_oracle.iface(1), cfg)
    try:
        x, f0, style, _ = inputs(cfg, 17, 0)  # above max_frames
        with pytest.raises(RuntimeError):
            k.run(x, f0, style)
    finally:
        k.close()


def test_kokoro_generator_fusion_coverage():
    """The HIP planner's view of the generator graph (no device needed): every AdaIN1d (+ snake)
    and conv_1d chain collapses into one item (TTS_FUSE_ADAIN / TTS_FUSE_CONV)."""
    cfg = ttship.kokoro_gen_config(in_channels=64, style_dim=16, max_frames=16)
    k = ttship.KokoroGenerator(py_oracle.iface(4), cfg)
    try:
        k.run(*inputs(cfg, 4, 0))
        st = k.plan_stats()
        off = k.plan_stats(0)
    finally:
        k.close()
    n_adain = cfg.n_ups * (1 + cfg.n_kernels) * 3 * 2  # (noise + res blocks) x 3 units x 2 halves
    assert st["adain"] == n_adain
    assert st["conv"] >= n_adain  # every res-block conv (+ noise / post convs when they fit)
    assert st["unfused"] < off["unfused"] // 10
