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
@pytest.mark.parametrize("K,N", [(2048, 2048), (2048, 512), (8192, 64), (1024, 1024), (64, 7)])
@pytest.mark.parametrize("M", [1, 2, 8])
def test_q8_0(hip, K, N, M):
    rng = np.random.default_rng(K + N * 3 + M)
    w = helpers.rand_q8_0(rng, N, K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    ref = py_oracle.gemv(ttship.Q8_0, w, x, N)
    got = run_gpu(hip, ttship.Q8_0, w, x, N)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), np.abs(got - ref).max()  # exact ggml order


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
