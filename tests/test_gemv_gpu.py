"""Parity of the HIP dequant-GEMV (k_gemv.hip) against the CPU oracle (ggml-cpu semantics).

Bar: ggml's integer block dots are exact on both sides; only the f32 order of adding block terms
differs, so |gpu - oracle| <= 2e-6 * sum_k |w_k x_k| (F32/F16: f64 accumulation on both sides).
"""
import ctypes

import numpy as np
import pytest

import helpers
import py_oracle
import ttship

SHAPES = [(1024, 1024), (4096, 1024), (1024, 4096), (2048, 512), (3072, 1088), (256, 3)]


def run_gpu(hip, wtype, w, x, N):
    M, K = x.shape
    if wtype == ttship.Q4_K:  # the raw GEMV entry takes the backend's Q4_K lane layout
        w = np.ascontiguousarray(w, dtype=np.uint8)
        rp = np.empty_like(w)
        ttship.lib().tts_repack_q4_K(w.ctypes.data, rp.ctypes.data, w.nbytes // 144, 0)
        back = np.empty_like(w)
        ttship.lib().tts_repack_q4_K(rp.ctypes.data, back.ctypes.data, w.nbytes // 144, 1)
        assert np.array_equal(back, w)
        w = rp
    dw = hip.alloc(w.nbytes)
    dx = hip.alloc(x.nbytes)
    dy = hip.alloc(4 * M * N)
    try:
        hip.set(dw, w)
        hip.set(dx, x)
        st = ttship.lib().tts_hip_gemv(hip.ptr, wtype, dw, dx, dy, K, N, M)
        assert st == 0
        y = np.empty((M, N), dtype=np.float32)
        hip.get(y, dy)
        return y
    finally:
        hip.free(dw)
        hip.free(dx)
        hip.free(dy)


def magnitude(wdq, x):
    return np.abs(x.astype(np.float64)) @ np.abs(wdq.astype(np.float64)).T


@pytest.mark.gpu
@pytest.mark.parametrize("K,N", SHAPES)
@pytest.mark.parametrize("M", [1, 2, 5, 8, 11])
def test_q4_K(hip, K, N, M):
    if K % 256:
        pytest.skip("Q4_K needs K % 256 == 0")
    rng = np.random.default_rng(K * 7 + N + M)
    w = helpers.rand_q4_K(rng, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
    got = run_gpu(hip, ttship.Q4_K, w, x, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()  # exact ggml order


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("K,N", [(1024, 1024), (1024, 3072), (2048, 160), (3072, 512), (4096, 1024), (1024, 1000)])
@pytest.mark.parametrize("M", [9, 16, 17, 100, 448])
def test_q4_K_prefill_gemm(hip, tiled, K, N, M):
    """Many-column Q4_K products (prompt prefill): the operand pass over all columns, then the K-relay
    kernel over (16-row tile, 16-column tile) pairs, on lane-layout and tile-layout weights; N = 1000
    (not whole tiles) falls back to the 8-column GEMV loop.  Bit-identical to ggml's order."""
    rng = np.random.default_rng(K * 13 + N + M + tiled)
    w = helpers.rand_q4_K(rng, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
    got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("K,N,M", [(4096, 1024, 32), (2048, 160, 17), (4096, 512, 64)])
def test_q4_K_prefill_gemm_eight_waves(hip, tiled, K, N, M):
    """The many-column K-relay GEMM with a tile's blocks over eight waves (TTS_HIP_OPT_GEMM_KR_NW = 8,
    K >= 2048): the relay hands ggml's chain through eight waves in block order, bit-identical."""
    hip.set_option(ttship.OPT["GEMM_KR_NW"], 8)
    try:
        rng = np.random.default_rng(K * 5 + N + M + tiled)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        hip.set_option(ttship.OPT["GEMM_KR_NW"], 4)


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("K,N,M", [(1024, 1024, 32), (1024, 3072, 17), (2048, 160, 48), (1024, 4096, 64), (2048, 512, 100),
                                   (1024, 64, 448), (4096, 1024, 32)])
def test_q4_K_prefill_gemm_two_column_tiles(hip, tiled, K, N, M):
    """The many-column K-relay GEMM with two 16-column tiles per workgroup (TTS_HIP_OPT_GEMM_KR_CT2, K <=
    2048: the weight tile loaded once, both tiles' operands in LDS; K = 4096 keeps one tile): bit-identical."""
    hip.set_option(ttship.OPT["GEMM_KR_CT2"], 1)
    try:
        rng = np.random.default_rng(K * 3 + N + M + tiled)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        hip.set_option(ttship.OPT["GEMM_KR_CT2"], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("opt,val", [("GEMM_KR_CP", 1), ("GEMM_KR_XCD", 1)])
@pytest.mark.parametrize("K,N,M", [(1024, 1024, 32), (2048, 1024, 32), (1024, 3072, 48), (2048, 160, 17), (1024, 512, 64),
                                   (4096, 1024, 32)])
def test_q4_K_prefill_gemm_column_pairs(hip, tiled, opt, val, K, N, M):
    """The many-column K-relay GEMM with a row tile's two column tiles on one workgroup's two wave halves
    (TTS_HIP_OPT_GEMM_KR_CP; K = 4096 keeps one tile per workgroup), and with the XCD-contiguous
    column-tile order (TTS_HIP_OPT_GEMM_KR_XCD = 1; off by default): the same sums, bit-identical (odd
    tile counts leave the last pair's second half idle)."""
    dflt = {"GEMM_KR_CP": 0, "GEMM_KR_XCD": 0}[opt]
    hip.set_option(ttship.OPT[opt], val)
    try:
        rng = np.random.default_rng(K * 5 + N + M + tiled)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        hip.set_option(ttship.OPT[opt], dflt)


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("K,N,M", [(1024, 1024, 64), (4096, 1024, 80), (2048, 512, 100), (3072, 256, 77), (1024, 3072, 576),
                                   (1024, 48, 65), (4096, 16, 130)])
@pytest.mark.parametrize("nw", [4, 8])
def test_q4_K_prefill_gemm_pf(hip, tiled, K, N, M, nw):
    """The prompt pass's Q4_K GEMM (k_gemm_q4K_pf, TTS_HIP_OPT_GEMM_PF: >= 64 columns by default): a wave per
    two 16-row tiles of one 16-column tile over the whole row, ggml's block chain in registers -- the same
    sums in the same order as the oracle, bit-identical (ragged last column tiles, row counts that leave
    a workgroup's last waves without a tile)."""
    hip.set_option(ttship.OPT["GEMM_PF"], 64)
    hip.set_option(ttship.OPT["GEMM_PF_NW"], nw)
    try:
        rng = np.random.default_rng(K * 11 + N + M + tiled)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        hip.set_option(ttship.OPT["GEMM_PF_NW"], 4)


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("walk", [3, 8])
@pytest.mark.parametrize("K,N,M", [(1024, 1024, 96), (4096, 1024, 80), (2048, 512, 100), (3072, 256, 77), (1024, 3072, 576)])
def test_q4_K_prefill_gemm_row_walk(hip, tiled, walk, K, N, M):
    """The prompt pass's many-column K-relay GEMM with `walk` workgroups per column tile, each copying its
    operand tile once and walking every walk-th row tile (TTS_HIP_OPT_GEMM_KR_WALK; more than 4 column
    tiles): the same sums, bit-identical."""
    hip.set_option(ttship.OPT["GEMM_KR_WALK"], walk)
    try:
        rng = np.random.default_rng(K * 3 + N + M + tiled + walk)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        hip.set_option(ttship.OPT["GEMM_KR_WALK"], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("K,N,M", [(1024, 1024, 32), (4096, 1024, 32), (1024, 3072, 9), (2048, 160, 17), (4096, 512, 64),
                                   (3072, 256, 40)])
def test_q4_K_prefill_gemm_in_kernel_operands(hip, tiled, K, N, M):
    """The many-column K-relay GEMM without the operand pass (TTS_HIP_OPT_GEMM_KR_INKERNEL): each (row
    tile, column tile) workgroup quantizes its own 16 columns; the same operands, bit-identical."""
    hip.set_option(ttship.OPT["GEMM_KR_INKERNEL"], 64)
    try:
        rng = np.random.default_rng(K * 7 + N + M + tiled)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu_tiled(hip, w, x, N) if tiled else run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        hip.set_option(ttship.OPT["GEMM_KR_INKERNEL"], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,M", [(1024, 64, 12000), (4096, 32, 3000)])
def test_q4_K_prefill_gemm_column_chunks(hip, K, N, M):
    """A prompt pass over many prompts (64 prompts x 448 tokens) has more columns than the 64 MiB operand
    area holds: the GEMM runs in passes over column chunks of whole 16-column tiles, bit-identical."""
    rng = np.random.default_rng(K + N + M)
    w = helpers.rand_q4_K(rng, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
    got = run_gpu(hip, ttship.Q4_K, w, x, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()


Q80_PATHS = {"slab_pro": (1, 1, 0), "slab": (1, 0, 0), "rows_pro": (0, 1, 0), "rows": (0, 0, 0), "slab_rw1": (1, 1, 1),
             "slab_rw32": (1, 0, 32)}


@pytest.mark.gpu
@pytest.mark.parametrize("path", list(Q80_PATHS))
@pytest.mark.parametrize("K,N", [(2048, 2048), (2048, 512), (8192, 64), (1024, 1024), (64, 7), (768, 33), (4096, 1000)])
@pytest.mark.parametrize("M", [1, 2, 3, 8, 9, 64, 300])
def test_q8_0(hip, path, K, N, M):
    """M > 8: the int8 matrix-core GEMM (k_gemm_q8_0): per-block exact int dots, ggml's f32 chain.
    M <= 8, K % 256 == 0: the slab kernel (TTS_HIP_OPT_GEMV_Q80_SLAB = 1; rows per workgroup auto, 1 or
    32, partial last workgroups) or the (row, block)-per-thread kernel, each with the activation quantized
    to Q8_0 inside every workgroup (TTS_HIP_OPT_GEMV_Q80_PRO = 1: quantize_row_q8_0 per 32 elements) or by
    the separate quantize launch."""
    slab, pro, rw = Q80_PATHS[path]
    if M > 8 and path != "slab_pro":
        pytest.skip("M > 8 runs the matrix-core GEMM on every path")
    lib = ttship.lib()
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_PRO"], pro) == 0
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_SLAB"], slab) == 0
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_RW"], rw) == 0
    try:
        rng = np.random.default_rng(K + N * 3 + M)
        w = helpers.rand_q8_0(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        x[0, :32] = 0.0  # an all-zero block: d = 0, id = 0
        ref = py_oracle.gemv(ttship.Q8_0, w, x, N)
        got = run_gpu(hip, ttship.Q8_0, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()  # exact ggml order
    finally:
        lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_PRO"], 1)
        lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_SLAB"], 1)
        lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_RW"], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("staged", [2, 1, 0])
@pytest.mark.parametrize("K,N", [(1024, 1024), (4096, 1024), (1024, 4096), (2048, 200), (256, 64), (8192, 96), (96, 40)])
@pytest.mark.parametrize("M", [9, 64, 130, 1000])
def test_q8_0_gemm(hip, staged, K, N, M):
    """Many-column Q8_0 products (Dia's encoder, prefills) on the int8 matrix cores: the staged kernel
    (TTS_HIP_OPT_GEMM_Q8_STAGED = 2: 64 x 128 output tiles, 1: 64 x 64; operands of 8 blocks per stage
    through two LDS buffers) and the direct-load kernel (0; also K % 256 != 0).  Partial row and column
    tiles.  Bit-identical to ggml's block order."""
    lib = ttship.lib()
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMM_Q8_STAGED"], staged) == 0
    try:
        rng = np.random.default_rng(K * 7 + N * 3 + M + staged)
        w = helpers.rand_q8_0(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        x[1, 32:64] = 0.0
        ref = py_oracle.gemv(ttship.Q8_0, w, x, N)
        got = run_gpu(hip, ttship.Q8_0, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMM_Q8_STAGED"], 2)


@pytest.mark.gpu
@pytest.mark.parametrize("wtype", [ttship.F32, ttship.F16])
@pytest.mark.parametrize("K,N", [(1024, 1088), (768, 768), (640, 1024), (4, 9)])
@pytest.mark.parametrize("M", [1, 3, 9])
def test_float(hip, wtype, K, N, M):
    rng = np.random.default_rng(K + N + M + wtype)
    wf = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
    w = wf.astype(np.float16) if wtype == ttship.F16 else wf
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = py_oracle.gemv(wtype, w.view(np.uint8), x, N)
    got = run_gpu(hip, wtype, w.view(np.uint8), x, N)
    # f64 accumulation on both sides: agreement to the final f32 rounding
    helpers.assert_close_scaled(got, ref, magnitude(w.astype(np.float32), x), 1e-7, "float")


MF_SHAPES = [(1024, 1024), (256, 4), (1024, 1000), (3072, 2048), (8192, 512), (4096, 1024), (3072, 8192)]


def run_gpu_tiled(hip, w, x, N):
    """Raw GEMV on a weight in the backend's 4-row tile layout (the matrix-core kernel)."""
    M, K = x.shape
    w = np.ascontiguousarray(w, dtype=np.uint8)
    tl = np.empty_like(w)
    ttship.lib().tts_repack_q4_K_tiled(w.ctypes.data, tl.ctypes.data, N, K // 256, 0)
    dw = hip.alloc(tl.nbytes)
    dx = hip.alloc(x.nbytes)
    dy = hip.alloc(4 * M * N)
    try:
        hip.set(dw, tl)
        hip.set(dx, x)
        assert ttship.lib().tts_hip_gemv_ex(hip.ptr, ttship.Q4_K, dw, dx, dy, K, N, M, 32) == 0  # TTS_FLAG_TILED
        y = np.empty((M, N), dtype=np.float32)
        hip.get(y, dy)
        return y
    finally:
        hip.free(dw)
        hip.free(dx)
        hip.free(dy)


KS_DEFAULT = 256  # backend default of TTS_HIP_OPT_GEMV_KS


# (GEMV_KS tile cap, GEMV_KRELAY, GEMV_PREQUANT, GEMV_KR_INKERNEL)
MF_PATHS = {"mf": (0, 0, 1, 0), "ks": (KS_DEFAULT, 0, 1, 0), "ks_loop": (1 << 20, 0, 1, 0), "kr": (KS_DEFAULT, 1, 1, 0),
            "kr_inkernel": (KS_DEFAULT, 1, 1, 4096), "mf_inkernel": (0, 0, 0, 0), "ks_inkernel": (KS_DEFAULT, 0, 0, 0)}


@pytest.fixture(params=list(MF_PATHS), ids=list(MF_PATHS))
def ks_tiles(request, hip):
    """Tile-layout GEMVs on k_gemv_q4K_mf, on the K-split kernel k_gemv_q4K_ks where it applies
    (M <= 8, K <= 4096, N % 16 == 0) with the default tile cap and for every tile count (grids of more
    than 2048 tiles loop over tiles), on the K-relay kernel k_gemv_q4K_kr (M <= 8, K = 1024 * {1, 2,
    3, 4, 8}, N % 16 == 0; the default), each after the quantize pass (k_quant_mf, default) or with
    the operands quantized inside every workgroup (for the K relay: K <= 4096)."""
    lib = ttship.lib()
    ks, kr, pre, ink = MF_PATHS[request.param]
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_KS"], ks) == 0
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_KRELAY"], kr) == 0
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_PREQUANT"], pre) == 0
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_KR_INKERNEL"], ink) == 0
    yield request.param
    lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_KS"], KS_DEFAULT)
    lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_KRELAY"], 1)
    lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_PREQUANT"], 1)
    lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_KR_INKERNEL"], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N", MF_SHAPES + [(8192, 3072), (3072, 16388), (3072, 40960), (256, 48)])
@pytest.mark.parametrize("M", [1, 2, 5, 8, 16, 19])
def test_q4_K_mfma(hip, ks_tiles, K, N, M):
    """Matrix-core Q4_K paths on the tile layout (k_gemv_q4K_mf; k_gemv_q4K_ks): the integer block
    dots run as f16 MFMAs whose sums are exact integers, and ggml's f32 chain runs in block order,
    so the result is bit-identical to ggml's order."""
    rng = np.random.default_rng(K * 5 + N + 3 * M)
    w = helpers.rand_q4_K(rng, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
    got = run_gpu_tiled(hip, w, x, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()


@pytest.mark.gpu
def test_q4_K_mfma_extreme_blocks(hip, ks_tiles):
    """Largest integer sums the MFMA path must keep exact: all scales / mins 63, nibbles 15, and
    activations quantized to +-127 (|aux32| up to 3.84e6, bsum up to 4064)."""
    K, N, M = 1024, 64, 4
    rng = np.random.default_rng(7)
    w = helpers.rand_q4_K(rng, N, K)
    blk = w.reshape(-1, 144)
    blk[:, 4:16] = 0xFF               # every 6-bit scale and min = 63
    blk[: len(blk) // 2, 16:] = 0xFF  # nibbles 15
    x = np.full((M, K), 3.0, dtype=np.float32)
    x[1] = -3.0
    x[2, ::2] = -1.0
    x[3] = rng.standard_normal(K).astype(np.float32)
    ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
    got = run_gpu_tiled(hip, w, x, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()


KS_SHAPES = [(4096, 1024), (2048, 1024), (3072, 1024), (2560, 3072), (4096, 40), (8192, 100)]


@pytest.mark.gpu
@pytest.mark.parametrize("ks", [0, 1])
@pytest.mark.parametrize("K,N", KS_SHAPES)
@pytest.mark.parametrize("M", [1, 3, 5, 8])
def test_q4_K_unique(hip, ks, K, N, M):
    """Lane-layout Q4_K GEMV on the unique-load kernel (TTS_HIP_OPT_GEMV_UNIQUE = 1: an octet per
    (row, block), ggml's chain finished in block order from LDS) and on the octet-per-(row, column)
    kernel (0): both bit-identical to ggml's sequential order.  nb = 10 and 12 leave octets idle."""
    lib = ttship.lib()
    assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_UNIQUE"], ks) == 0
    try:
        rng = np.random.default_rng(K * 3 + N + 11 * M + ks)
        w = helpers.rand_q4_K(rng, N, K)
        x = rng.standard_normal((M, K)).astype(np.float32)
        ref = py_oracle.gemv(ttship.Q4_K, w, x, N)
        got = run_gpu(hip, ttship.Q4_K, w, x, N)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()
    finally:
        lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_UNIQUE"], 1)
