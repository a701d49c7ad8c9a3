"""Codec convolutions on the HIP backend vs the CPU oracle.

These ops are floating point with a different accumulation on each side (oracle: f64 sums, as
ggml's generic dot; GPU: f32 MFMA / FMA accumulation), so the bar is a relative tolerance, 1e-5 of
the output's scale -- far inside the PCM bar (1e-4 absolute) the codec tests check end to end.
im2col is a pure gather + fp16 rounding and must be bit-exact; the MFMA lane mapping is checked
bit-exactly with small-integer data (exact in f32 whatever the order).
"""
import numpy as np
import pytest

import convs
import nodes as nd
import ttship

F32, F16 = ttship.F32, ttship.F16


def run_both(hip, build):
    g1, g2 = nd.Graph(), nd.Graph()
    o1, o2 = build(g1), build(g2)
    g1.run_hip(hip)
    g2.run_oracle()
    return [(g1.node_array(a), g2.node_array(b)) for a, b in zip(o1, o2)]


def rnd(seed, *shape, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


def assert_rel(gpu, ref, rel=1e-5):
    scale = max(float(np.max(np.abs(ref))), 1e-30)
    err = float(np.max(np.abs(gpu.astype(np.float64) - ref.astype(np.float64))))
    assert err <= rel * scale, f"max err {err:.3e} vs scale {scale:.3e}"


CT_CASES = [  # IC, OC, L, K, s, p, d, op, groups
    (8, 4, 5, 16, 8, 4, 1, 0, 1),       # DAC upsampler shape (K = 2s)
    (96, 48, 40, 16, 8, 4, 1, 0, 1),    # DAC-like channel counts
    (64, 32, 33, 4, 2, 1, 1, 0, 1),     # DAC last stage (s = 2)
    (6, 6, 7, 3, 2, 1, 1, 1, 6),        # Kokoro depthwise (2,1,1,1,C)
    (16, 8, 12, 20, 10, 5, 1, 0, 1),    # Kokoro generator (stride 10)
    (64, 32, 40, 20, 10, 5, 1, 0, 1),   # Kokoro ups[0] shape, LDS polyphase kernel (S = 10)
    (32, 16, 70, 12, 6, 3, 1, 0, 1),    # Kokoro ups[1] shape, LDS polyphase kernel (S = 6)
    (5, 3, 4, 3, 3, 2, 2, 1, 1),        # dilated
]


@pytest.mark.gpu
@pytest.mark.parametrize("wtype", [F32, F16])
@pytest.mark.parametrize("case", CT_CASES)
def test_conv_transpose_1d(hip, case, wtype):
    IC, OC, L, K, s, p, d, op, grp = case
    x = rnd(1, IC, L)
    w = rnd(2, IC, OC // grp, K, scale=0.2)
    (gpu, ref), = run_both(hip, lambda g: [convs.conv_transpose_1d(g, x, w, s, p, d, op, grp, wtype)])
    assert_rel(gpu, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(16, 12, 40, 7, 1, 9, 3), (8, 64, 33, 1, 1, 0, 1), (64, 96, 300, 7, 1, 3, 1), (96, 1, 100, 7, 1, 3, 1),
                                  (22, 16, 241, 1, 1, 0, 1), (22, 32, 241, 12, 6, 3, 1), (9, 24, 500, 11, 1, 25, 5)])
def test_conv_1d(hip, case):
    IC, OC, L, K, s, p, d = case
    x = rnd(3, IC, L)
    w = rnd(4, OC, IC, K, scale=0.1)
    (gpu, ref), = run_both(hip, lambda g: [convs.conv_1d(g, x, w, s, p, d)])
    assert_rel(gpu, ref)


@pytest.mark.gpu
def test_im2col_bit_exact(hip):
    IC, L, K, s, p, d = 24, 57, 7, 1, 9, 3
    x = rnd(5, IC, L, scale=3.0)
    w = rnd(6, 1, IC, K)

    OL = (L + 2 * p - d * (K - 1) - 1) // s + 1
    g1, g2 = nd.Graph(), nd.Graph()
    o1, o2 = [g.node("IM2COL", F16, [IC * K, OL, 1], [g.leaf(w), g.leaf(x)], params=[s, 1, p, 0, d, 1, 0]) for g in (g1, g2)]
    g1.run_hip(hip)
    g2.run_oracle()
    gpu, ref = g1.node_array(o1, dtype=np.float16), g2.node_array(o2, dtype=np.float16)
    assert np.array_equal(gpu.view(np.uint16), ref.view(np.uint16))


@pytest.mark.gpu
@pytest.mark.parametrize("wtype", [F32, F16])
def test_gemm_mfma_integer_exact(hip, wtype):
    """Small integers: every product and partial sum is exact in f32, so any correct lane
    mapping gives the oracle's bits; an asymmetric B catches a transposed store."""
    rng = np.random.default_rng(7)
    IC, OC, L, K = 40, 37, 70, 3
    x = rng.integers(-3, 4, size=(IC, L)).astype(np.float32)
    w = (rng.integers(-4, 5, size=(OC, IC, K)) + np.arange(OC)[:, None, None] * 0.25).astype(np.float32)
    (gpu, ref), = run_both(hip, lambda g: [convs.conv_1d(g, x, w, 1, 1, 1, wtype=wtype)])
    assert np.array_equal(gpu, ref)


CONV_EPI_CASES = [  # IC, OC, L, K, s, p, d, bias, residual
    (64, 64, 300, 7, 1, 9, 3, True, True),     # DAC residual unit (dilated k7) + bias + skip
    (128, 128, 241, 11, 1, 25, 5, True, True),  # Kokoro level-1 res block conv (k11, d5)
    (22, 256, 241, 12, 6, 3, 1, True, False),   # Kokoro noise conv (stride 6) + bias
    (22, 128, 241, 1, 1, 0, 1, True, False),    # Kokoro 1-tap noise conv over 22 STFT channels
    (96, 1, 100, 7, 1, 3, 1, True, False),      # DAC output conv (one channel)
    (8, 70, 33, 1, 1, 0, 1, False, False),      # quantizer out_proj (no epilogue)
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CONV_EPI_CASES)
def test_conv_1d_fused_epilogue(hip, case):
    """IM2COL -> MUL_MAT -> ADD bias -> ADD residual as one implicit-GEMM kernel (TTS_FUSE_CONV)
    against the unfused node chain and the oracle: the f64 sums differ only in order, so the f32
    results agree bit for bit except at f64 near-ties."""
    IC, OC, L, K, s, p, d, with_bias, with_res = case
    x = rnd(5, IC, L)
    w = rnd(6, OC, IC, K, scale=0.1)
    b = rnd(7, OC, 1)
    OL = (L + 2 * p - d * (K - 1) - 1) // s + 1
    r = rnd(8, OC, OL)

    def build(g):
        y = convs.conv_1d(g, x, w, s, p, d)
        if with_bias:
            y = g.node("ADD", F32, [OL, OC], [y, g.leaf(b)])
        if with_res:
            y = g.node("ADD", F32, [OL, OC], [g.leaf(r), y])
        return [y]
    (fused, ref), = run_both(hip, build)
    hip.set_option(0, ttship.FUSE_ALL & ~ttship.FUSE["CONV"])
    try:
        (plain, _), = run_both(hip, build)
    finally:
        hip.set_option(0, ttship.FUSE_ALL)
    for got in (fused, plain):
        assert got.shape == ref.shape
        assert float(np.mean(got != ref)) <= 1e-3
        assert_rel(got, ref, rel=1e-6)
