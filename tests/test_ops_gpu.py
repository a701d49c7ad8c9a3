"""Op-level parity: each ggml op node run on the HIP backend and on the CPU oracle from the same
inputs.  Bar: bit-exact (the kernels reproduce ggml-cpu's f32 operation order; reductions ggml
performs in f64 are f64 on both sides; transcendentals are correctly rounded on both sides).
"""
import numpy as np
import pytest

import nodes as nd
import ttship

F32 = ttship.F32


def run_both(hip, build):
    """build(g) -> list of output tensors; returns [(gpu, oracle)] arrays."""
    g1, g2 = nd.Graph(), nd.Graph()
    o1, o2 = build(g1), build(g2)
    g1.run_hip(hip)
    g2.run_oracle()
    return [(g1.node_array(a), g2.node_array(b)) for a, b in zip(o1, o2)]


def assert_bits(pairs, what):
    for k, (a, b) in enumerate(pairs):
        if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
            d = np.abs(a.astype(np.float64) - b)
            raise AssertionError(f"{what}[{k}]: {np.sum(a != b)} / {a.size} differ, max {np.nanmax(d):.3e}")


def rnd(seed, *shape, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 1, 1024), (3, 6, 256), (2, 5, 768), (1, 7, 3)])
@pytest.mark.parametrize("op", ["NORM", "RMS_NORM"])
def test_norms(hip, shape, op):
    x = rnd(1, *shape) + 0.25

    def build(g):
        a = g.leaf(x)
        return [g.node(op, F32, list(x.shape[::-1]), [a], fparams={0: 1e-5})]
    assert_bits(run_both(hip, build), op)


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["ADD", "SUB", "MUL", "DIV"])
@pytest.mark.parametrize("bshape", [(3, 6, 256), (1, 1, 256), (6, 1), (1,)])
def test_binary_broadcast(hip, op, bshape):
    a = rnd(2, 3, 6, 256)
    full = (1,) * (3 - len(bshape)) + tuple(bshape)
    if full[-1] == 1 and len(bshape) == 1:
        full = (1, 1, 1)
    b = rnd(3, *full) + 2.0

    def build(g):
        ta, tb = g.leaf(a), g.leaf(b)
        return [g.node(op, F32, list(a.shape[::-1]), [ta, tb])]
    assert_bits(run_both(hip, build), op)


@pytest.mark.gpu
@pytest.mark.parametrize("uop", ["GELU", "SILU", "TANH", "SIGMOID", "EXP", "ABS", "NEG", "RELU"])
def test_unary(hip, uop):
    x = rnd(4, 7, 333, scale=3.0)

    def build(g):
        a = g.leaf(x)
        return [g.node("UNARY", F32, list(x.shape[::-1]), [a], params=[ttship.UNARY[uop]])]
    assert_bits(run_both(hip, build), uop)


@pytest.mark.gpu
@pytest.mark.parametrize("op,fp", [("SCALE", {0: 0.37}), ("SQR", {}), ("SQRT", {}), ("SIN", {}), ("COS", {}),
                                   ("CLAMP", {0: -0.5, 1: 0.75}), ("LEAKY_RELU", {0: 0.2}), ("ROUND", {}),
                                   ("MOD", {0: 1.0})])
def test_map_ops(hip, op, fp):
    x = rnd(5, 5, 129, scale=4.0)
    if op == "SQRT":
        x = np.abs(x)

    def build(g):
        a = g.leaf(x)
        return [g.node(op, F32, list(x.shape[::-1]), [a], fparams=fp)]
    assert_bits(run_both(hip, build), op)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,nc,heads,masked", [(1, 77, 16, True), (4, 77, 16, True), (3, 450, 8, False), (1, 4096, 2, True)])
def test_soft_max(hip, rows, nc, heads, masked):
    x = rnd(6, heads, rows, nc, scale=3.0)
    m = np.zeros((rows, nc), dtype=np.float32)
    m[:, nc // 2:] = -np.inf if rows > 1 else 0.0

    def build(g):
        a = g.leaf(x)
        srcs = [a, g.leaf(m)] if masked else [a]
        return [g.node("SOFT_MAX", F32, list(x.shape[::-1]), srcs, fparams={0: 0.125, 1: 0.0})]
    assert_bits(run_both(hip, build), "soft_max")


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,M,B", [(64, 450, 1, 16), (450, 1, 64, 16), (128, 33, 2, 4),
                                     (128, 1024, 1024, 2), (1024, 128, 1024, 2), (64, 448, 448, 3), (37, 70, 19, 2)])
def test_mul_mat_f32_batched(hip, K, N, M, B):
    """3-D float products: decode shapes on the generic kernel, many-query shapes (Dia's encoder
    attention, prompt prefill) on the tiled batched GEMM; both bit-identical to the oracle."""
    a = rnd(7, B, N, K)
    b = rnd(8, B, M, K)

    def build(g):
        ta, tb = g.leaf(a), g.leaf(b)
        return [g.node("MUL_MAT", F32, [N, M, B], [ta, tb])]
    assert_bits(run_both(hip, build), "mul_mat")


@pytest.mark.gpu
def test_mul_mat_f32_batched_broadcast(hip):
    """src0 broadcast over src1's batch dims (GQA-style: r2 = 4, r3 = 2)."""
    K, N, M = 64, 40, 48
    a = rnd(31, 1, 2, N, K)
    b = rnd(32, 2, 8, M, K)

    def build(g):
        return [g.node("MUL_MAT", F32, [N, M, 8, 2], [g.leaf(a), g.leaf(b)])]
    assert_bits(run_both(hip, build), "mul_mat broadcast")


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,M", [(1090, 1024, 332), (46, 319, 640), (768, 768, 64), (640, 256, 9), (33, 70, 100), (2048, 768, 17)])
@pytest.mark.parametrize("epi", [None, "GELU", "ADD"])
def test_mul_mat_f32_gemm(hip, K, N, M, epi):
    """2-D float MUL_MATs with more than 8 columns run on the tiled GEMM (k_gemm.hip), through the
    planner's GEMV items (<= 64 columns, with their fused GELU / residual epilogues) or the plain op
    path; sequential f64 sums, so bit-identical to the oracle."""
    a = rnd(11, N, K, scale=0.2)
    b = rnd(12, M, K)
    r = rnd(13, M, N)

    def build(g):
        mm = g.node("MUL_MAT", F32, [N, M], [g.leaf(a), g.leaf(b)])
        if epi == "GELU":
            return [g.node("UNARY", F32, [N, M], [mm], params=[5])]
        if epi == "ADD":
            return [g.node("ADD", F32, [N, M], [mm, g.leaf(r)])]
        return [mm]
    assert_bits(run_both(hip, build), f"gemm {epi}")


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,M", [(1024, 9792, 32), (1024, 2176, 9), (1000, 4100, 16), (1024, 3000, 17), (512, 2048, 33),
                                   (1024, 2304, 64), (130, 5000, 24)])
@pytest.mark.parametrize("epi", [None, "GELU", "ADD"])
def test_mul_mat_f32_wide(hip, K, N, M, epi):
    """Many-row float MUL_MATs with 9..64 columns (the output heads of a 32-prompt step) run the wide
    GEMV (k_gemv_f32_wide: one ascending-k f64 chain per output, ggml_vec_dot_f32's order), K tails and
    row remainders included: bit-identical to the oracle."""
    a = rnd(31, N, K, scale=0.2)
    b = rnd(32, M, K)
    r = rnd(33, M, N)

    def build(g):
        mm = g.node("MUL_MAT", F32, [N, M], [g.leaf(a), g.leaf(b)])
        if epi == "GELU":
            return [g.node("UNARY", F32, [N, M], [mm], params=[5])]
        if epi == "ADD":
            return [g.node("ADD", F32, [N, M], [mm, g.leaf(r)])]
        return [mm]
    assert_bits(run_both(hip, build), f"wide gemv {epi}")


@pytest.mark.gpu
def test_custom_maps(hip):
    """The reference's CPU callbacks restated on the device: cfg_scale (MAP_CUSTOM2, Dia) and
    uv_noise_compute (MAP_CUSTOM3, Kokoro, host draws and device-hashed draws)."""
    c, u = rnd(21, 3, 2, 1028), rnd(22, 3, 2, 1028)
    L, H = 900, 9
    f0 = np.abs(rnd(23, L)) * 20.0  # some below the voicing threshold 10
    data = np.concatenate([np.array([10.0, 0.003, 0.1, np.float32(0.1) / np.float32(3)], np.float32),
                           np.random.default_rng(24).random(L * H, dtype=np.float32)])

    def build(g):
        cfg = g.node("MAP_CUSTOM2", F32, [1028, 2, 3], [g.leaf(c), g.leaf(u)], params=[2], fparams={1: 3.0})
        uvn = g.node("MAP_CUSTOM3", F32, [L, H, 2], [g.leaf(np.zeros((2, H, L), np.float32)), g.leaf(f0), g.leaf(data)], params=[1])
        uvh = g.node("MAP_CUSTOM3", F32, [L, H, 2], [g.leaf(np.zeros((2, H, L), np.float32)), g.leaf(f0), g.leaf(data[:4].copy())],
                     params=[1, 1, 0x1234, 0])
        return [cfg, uvn, uvh]
    pairs = run_both(hip, build)
    assert_bits(pairs, "custom maps")
    voiced = f0 > 10.0
    uv = pairs[1][1].reshape(2, H, L)
    assert np.all(uv[0][:, voiced] == np.float32(0.1)) and np.all(uv[0][:, ~voiced] == 0)
    assert 0.0 < float(pairs[2][1].reshape(2, H, L)[1].std()) < 0.1  # hashed draws present


@pytest.mark.gpu
def test_get_rows_and_concat_and_cpy(hip):
    tab = rnd(9, 40, 96)
    idx = np.array([3, 0, 39, 7, 7], dtype=np.int32)
    x = rnd(10, 4, 96)
    y = rnd(11, 2, 96)

    def build(g):
        t = g.leaf(tab)
        i = g.leaf(idx, typ=ttship.I32)
        gr = g.node("GET_ROWS", F32, [96, 5], [t, i])
        c = g.node("CONCAT", F32, [96, 6], [g.leaf(x), g.leaf(y)], params=[1])
        xt = g.leaf(x)
        tr = g.transpose(xt)
        ct = g.node("CONT", F32, [4, 96], [tr])
        return [gr, c, ct]
    assert_bits(run_both(hip, build), "get_rows/concat/cont")


@pytest.mark.gpu
def test_rope_neox_freq_factors(hip):
    x = rnd(12, 4, 3, 128)  # [T, H, hd] -> ggml ne [128, 3, 4]
    pos = np.array([0, 5, 17, 400], dtype=np.int32)
    ff = np.linspace(1.0, 8.0, 64).astype(np.float32)

    def build(g):
        tx, tp, tf = g.leaf(x), g.leaf(pos, typ=ttship.I32), g.leaf(ff)
        return [g.node("ROPE", F32, [128, 3, 4], [tx, tp, tf], params=[0, 128, 2, 0, 131072],
                       fparams={5: 500000.0, 6: 1.0, 7: 0.0, 8: 1.0})]
    assert_bits(run_both(hip, build), "rope")
