"""Kokoro sine-source / iSTFTNet-head ops on the HIP backend vs the CPU oracle.

Both sides run the same operation order (oracle/ggml_ref.c op_cumsum / op_upscale / op_stft /
op_istft, tts.cpp_amd/csrc/k_audio.hip), so CUMSUM and UPSCALE must be bit-exact.  STFT/ISTFT
evaluate atan2 / cos / sin of data in f64 through two different libms (glibc, ocml), which can
differ in the last f64 bit; after rounding to f32 that shows up at most as a 1-ulp difference in
rare elements, so those are held to <= 1 ulp with almost every element bit-exact.  The oracle
itself is pinned to float32 torch in tests/test_oracle_golden.py.
"""
import numpy as np
import pytest

import audio_ops as ao
import nodes as nd
import ttship

F32 = ttship.F32


def run_both(hip, build):
    g1, g2 = nd.Graph(), nd.Graph()
    o1, o2 = build(g1), build(g2)
    g1.run_hip(hip)
    g2.run_oracle(n_threads=8)
    return [(g1.node_array(a), g2.node_array(b)) for a, b in zip(o1, o2)]


def hann(N):
    return np.array([np.float32(np.sin(np.pi * i / N) ** 2) for i in range(N)], dtype=np.float32)


def assert_ulp(gpu, ref, max_ulp=1, max_frac=1e-4):
    assert gpu.shape == ref.shape
    d = ao.ulp_diff(gpu, ref)
    frac = float(np.mean(gpu != ref)) if gpu.size else 0.0
    assert d <= max_ulp and frac <= max_frac, f"max ulp {d}, mismatching fraction {frac:.2e}"


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(9, 23), (9, 1600), (2, 5000), (1, 1), (3, 4097)])
def test_cumsum_bit_exact(hip, shape):
    x = np.random.default_rng(1).random(shape, dtype=np.float32)
    (gpu, ref), = run_both(hip, lambda g: [ao.cumsum(g, x)])
    assert np.array_equal(gpu, ref)


@pytest.mark.gpu
def test_cumsum_of_transposed_view(hip):
    x = np.random.default_rng(2).random((40, 9), dtype=np.float32)

    def build(g):
        xl = g.leaf(x)
        return [ao.cumsum(g, g.transpose(xl))]
    (gpu, ref), = run_both(hip, build)
    assert np.array_equal(gpu, ref)
    assert np.array_equal(ref.reshape(9, 40), np.cumsum(x.T.astype(np.float64), 1).astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("T,s", [(23, 300), (1600, 300), (7, 2), (7, 5), (1, 300)])
def test_upscale_linear_bit_exact(hip, T, s):
    x = (np.random.default_rng(3).standard_normal((9, T)) * 100).astype(np.float32)
    (gpu, ref), = run_both(hip, lambda g: [ao.upscale(g, x, T * s, 1)])
    assert np.array_equal(gpu, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,ne0", [((1, 1600), 480000), ((3, 7), 21), ((2, 5), 17)])
def test_upscale_nearest_bit_exact(hip, shape, ne0):
    x = np.random.default_rng(4).standard_normal(shape).astype(np.float32)
    (gpu, ref), = run_both(hip, lambda g: [ao.upscale(g, x, ne0, 0)])
    assert np.array_equal(gpu, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,L,B,abs_angle", [(20, 5, 1200, 1, 1), (20, 5, 48000, 1, 1), (16, 4, 160, 2, 0), (15, 4, 97, 1, 1),
                                               (512, 128, 4096, 1, 1), (20, 5, 11, 1, 1)])
def test_stft(hip, N, H, L, B, abs_angle):
    x = (np.random.default_rng(5).standard_normal((B, L)) * 0.3).astype(np.float32)
    (gpu, ref), = run_both(hip, lambda g: [ao.stft(g, x, hann(N), N, H, abs_angle)])
    assert_ulp(gpu, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,F,B,abs_angle", [(20, 5, 97, 1, 1), (20, 5, 9601, 1, 1), (16, 4, 33, 2, 0), (15, 4, 20, 1, 1),
                                               (512, 128, 40, 1, 1), (20, 1, 300, 1, 1), (20, 5, 2, 1, 1)])
def test_istft(hip, N, H, F, B, abs_angle):
    rng = np.random.default_rng(6)
    K = N // 2 + 1
    mag = np.exp(rng.standard_normal((B, F, K)) * 0.5).astype(np.float32)
    pha = np.sin(rng.standard_normal((B, F, K)) * 2.0).astype(np.float32)
    z = np.stack([mag, pha]).astype(np.float32)
    (gpu, ref), = run_both(hip, lambda g: [ao.istft(g, z, hann(N), N, H, abs_angle)])
    assert_ulp(gpu, ref)


@pytest.mark.gpu
def test_kokoro_sine_source_chain(hip):
    """build_sin_gen's deterministic front (model.cpp:174-176) + the har STFT (model.cpp:199):
    repeat * harmonic norm -> mod 1 -> cumsum -> x600pi -> linear x300 -> sin -> STFT(20, 5)."""
    T = 160
    f0 = (np.random.default_rng(7).random((1, T)) * 300.0).astype(np.float32)
    hn = (np.arange(1, 10, dtype=np.float32) / np.float32(24000.0))[:, None].astype(np.float32)

    def build(g):
        x = g.leaf(f0)
        shape = g.leaf(np.zeros((9, T), dtype=np.float32))
        rep = g.node("REPEAT", F32, [T, 9], [x, shape])
        cur = g.node("MUL", F32, [T, 9], [rep, g.leaf(hn)])
        cur = g.node("MOD", F32, [T, 9], [cur], fparams={0: 1.0})
        cur = ao.cumsum(g, cur)
        cur = g.node("SCALE", F32, [T, 9], [cur], fparams={0: float(np.float32(600.0 * np.pi))})
        up = ao.upscale(g, cur, T * 300, 1)
        s = g.node("SIN", F32, [T * 300, 9], [up])
        row = g.view(s, [T * 300, 1, 1, 1], [4, 4 * T * 300, 4 * T * 300, 4 * T * 300])
        har = g.node("CONT", F32, [T * 300, 1], [row])
        return [up, s, ao.stft(g, har, hann(20), 20, 5, 1)]
    (u, ur), (s, sr), (st, str_) = run_both(hip, build)
    assert np.array_equal(u, ur)
    assert np.array_equal(s, sr)
    assert_ulp(st, str_)


def _snake_graph(g, x, alpha):
    """snake_1d (src/util.cpp:98-101) with reciprocal() as DIV of a broadcast 1.0 (util.cpp:86-94)."""
    T, C = x.shape[1], x.shape[0]
    xl, al = g.leaf(x), g.leaf(alpha.reshape(C, 1))
    one = g.leaf(np.ones((1, 1), np.float32))
    onev = g.view(one, [1, C, 1, 1], [4, 0, 0, 0])
    recip = g.node("DIV", F32, [1, C], [onev, al])
    m1 = g.node("MUL", F32, [T, C], [xl, al])
    s = g.node("SIN", F32, [T, C], [m1])
    q = g.node("SQR", F32, [T, C], [s])
    m2 = g.node("MUL", F32, [T, C], [q, recip])
    return g.node("ADD", F32, [T, C], [xl, m2])


@pytest.mark.gpu
@pytest.mark.parametrize("C,T", [(96, 4096), (7, 33), (1536, 16)])
@pytest.mark.parametrize("fused", [True, False])
def test_snake_bit_exact(hip, C, T, fused):
    rng = np.random.default_rng(C + T)
    x = (rng.standard_normal((C, T)) * 2).astype(np.float32)
    alpha = rng.uniform(0.5, 1.5, C).astype(np.float32)
    if not fused:
        hip.set_option(0, ttship.FUSE_ALL & ~128)
    try:
        (gpu, ref), = run_both(hip, lambda g: [_snake_graph(g, x, alpha)])
    finally:
        hip.set_option(0, ttship.FUSE_ALL)
    assert np.array_equal(gpu, ref)
    want = x.astype(np.float64) + np.sin(alpha[:, None].astype(np.float64) * x) ** 2 / alpha[:, None]
    assert np.max(np.abs(ref.reshape(C, T) - want)) < 1e-5 * np.max(np.abs(want))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(96, 4096), (5, 3), (64, 100)])
def test_row_broadcast_binary_bit_exact(hip, shape):
    """ADD / MUL / DIV of a [T, C] activation by a per-channel [1, C] vector (conv bias, alpha)."""
    C, T = shape
    rng = np.random.default_rng(T)
    x = rng.standard_normal((C, T)).astype(np.float32)
    b = (rng.standard_normal((C, 1)) + 3).astype(np.float32)

    def build(g):
        xl, bl = g.leaf(x), g.leaf(b)
        return [g.node(op, F32, [T, C], [xl, bl]) for op in ("ADD", "SUB", "MUL", "DIV")]
    for gpu, ref in run_both(hip, build):
        assert np.array_equal(gpu, ref)


def _adain_graph(g, x, gamma, beta, alpha, snake):
    """One AdaIN1d half of build_kokoro_generator_res_block (kokoro/model.cpp:142-146), then
    snake_1d: NORM over time, CONT(TRANSPOSE), x + x*gamma + beta, CONT(TRANSPOSE) back."""
    C, T = x.shape
    xl = g.leaf(x)
    n = g.node("NORM", F32, [T, C], [xl], fparams={0: 1e-5})
    c1 = g.node("CONT", F32, [C, T], [g.transpose(n)])
    gl, bl = g.leaf(gamma.reshape(C, 1).T.copy()), g.leaf(beta.reshape(C, 1).T.copy())  # ne [C, 1]
    m = g.node("MUL", F32, [C, T], [c1, gl])
    a1 = g.node("ADD", F32, [C, T], [c1, m])
    a2 = g.node("ADD", F32, [C, T], [a1, bl])
    c2 = g.node("CONT", F32, [T, C], [g.transpose(a2)])
    if not snake:
        return c2
    al = g.leaf(alpha.reshape(C, 1))
    one = g.leaf(np.ones((1, 1), np.float32))
    onev = g.view(one, [1, C, 1, 1], [4, 0, 0, 0])
    recip = g.node("DIV", F32, [1, C], [onev, al])
    m1 = g.node("MUL", F32, [T, C], [c2, al])
    s = g.node("SIN", F32, [T, C], [m1])
    q = g.node("SQR", F32, [T, C], [s])
    m2 = g.node("MUL", F32, [T, C], [q, recip])
    return g.node("ADD", F32, [T, C], [c2, m2])


@pytest.mark.gpu
@pytest.mark.parametrize("C,T", [(128, 4801), (256, 800), (7, 33), (16, 20000), (3, 65536)])
@pytest.mark.parametrize("snake", [True, False])
@pytest.mark.parametrize("fused", [True, False])
def test_adain_snake_bit_exact(hip, C, T, snake, fused):
    rng = np.random.default_rng(C * 7 + T)
    x = (rng.standard_normal((C, T)) * 3 + 1).astype(np.float32)
    gamma = (rng.standard_normal(C) * 0.2).astype(np.float32)
    beta = (rng.standard_normal(C) * 0.2).astype(np.float32)
    alpha = rng.uniform(0.5, 1.5, C).astype(np.float32)
    if not fused:
        hip.set_option(0, ttship.FUSE_ALL & ~ttship.FUSE["ADAIN"])
    try:
        (gpu, ref), = run_both(hip, lambda g: [_adain_graph(g, x, gamma, beta, alpha, snake)])
    finally:
        hip.set_option(0, ttship.FUSE_ALL)
    assert np.array_equal(gpu, ref)
