"""Known-answer tests pinning the oracle's quant formats and fp16 arithmetic (CPU only).

The reference holds no golden vectors; these KATs use hand-built blocks whose
dequantized values follow analytically from the ggml block definitions
(block_q4_K: d, dmin, 6-bit packed scales/mins, nibbles; block_q8_0: d, int8).
"""
import ctypes

import numpy as np
import pytest

import helpers
import py_oracle


def test_fp16_roundtrip_all_patterns():
    L = py_oracle.lib()
    h = np.arange(65536, dtype=np.uint16)
    ref = h.view(np.float16).astype(np.float32)
    got = np.array([L.ref_fp16_to_fp32(int(v)) for v in h[::7]], dtype=np.float32)
    r = ref[::7]
    finite = np.isfinite(r)
    assert np.array_equal(got[finite].view(np.uint32), r[finite].view(np.uint32))
    assert np.all(np.isnan(got[np.isnan(r)]))


def test_fp32_to_fp16_rne_matches_numpy():
    L = py_oracle.lib()
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.standard_normal(3000) * 10.0 ** rng.integers(-8, 5, 3000),
                        np.array([0.0, -0.0, 65504.0, 65520.0, 1e-8, 5.96e-8, 2.98e-8])]).astype(np.float32)
    got = np.array([L.ref_fp32_to_fp16(float(v)) for v in x], dtype=np.uint16)
    assert np.array_equal(got, x.astype(np.float16).view(np.uint16))


def _q4k_block(d, dmin, sc, mn, q):
    """Pack one Q4_K block exactly as quantize_row_q4_K_ref does."""
    b = np.zeros(144, dtype=np.uint8)
    b[0:2] = np.array([d], dtype=np.float16).view(np.uint8)
    b[2:4] = np.array([dmin], dtype=np.float16).view(np.uint8)
    s = np.zeros(12, dtype=np.uint8)
    for j in range(8):
        ls, lm = sc[j] & 63, mn[j] & 63
        if j < 4:
            s[j] = ls
            s[j + 4] = lm
        else:
            s[j + 4] = (ls & 0xF) | ((lm & 0xF) << 4)
            s[j - 4] |= (ls >> 4) << 6
            s[j] |= (lm >> 4) << 6
    b[4:16] = s
    qs = np.zeros(128, dtype=np.uint8)
    for c in range(4):
        for l in range(32):
            qs[32 * c + l] = q[64 * c + l] | (q[64 * c + 32 + l] << 4)
    b[16:] = qs
    return b


def test_q4_K_dequant_known_answer():
    rng = np.random.default_rng(7)
    sc = rng.integers(0, 64, 8)
    mn = rng.integers(0, 64, 8)
    q = rng.integers(0, 16, 256)
    d, dmin = 0.5, 0.25  # exactly representable in fp16
    blk = _q4k_block(d, dmin, sc, mn, q)
    got = py_oracle.dequant_q4_K(blk, 256, 1)[0]
    want = np.array([d * sc[i // 32] * q[i] - dmin * mn[i // 32] for i in range(256)], dtype=np.float64)
    assert np.array_equal(got.astype(np.float64), want)  # all values exact in f32


def test_q4_K_scale_packing_high_bits():
    # scales/mins >= 16 in sub-blocks 4..7 exercise the 2-bit high parts stored in bytes 0..7
    sc = np.array([63, 1, 2, 3, 48, 33, 63, 17])
    mn = np.array([0, 63, 5, 6, 60, 16, 31, 62])
    q = np.full(256, 15)
    blk = _q4k_block(1.0, 1.0, sc, mn, q)
    got = py_oracle.dequant_q4_K(blk, 256, 1)[0]
    for j in range(8):
        assert np.all(got[32 * j:32 * j + 32] == 15.0 * sc[j] - mn[j])


def test_q8_0_dequant_known_answer():
    blk = np.zeros(34, dtype=np.uint8)
    blk[0:2] = np.array([0.125], dtype=np.float16).view(np.uint8)
    q = np.arange(-16, 16, dtype=np.int8)
    blk[2:] = q.view(np.uint8)
    got = py_oracle.dequant_q8_0(blk, 32, 1)[0]
    assert np.array_equal(got, q.astype(np.float32) * 0.125)


def test_q8_K_quantize_properties():
    L = py_oracle.lib()
    rng = np.random.default_rng(3)
    x = rng.standard_normal(512).astype(np.float32)
    x[100] = -5.0  # signed max of block 0 is negative
    out = np.zeros(2 * 292, dtype=np.uint8)
    L.ref_quantize_row_q8_K(x.ctypes.data, out.ctypes.data, 512)
    for b in range(2):
        blk = out[b * 292:(b + 1) * 292]
        dq = blk[0:4].view(np.float32)[0]
        qs = blk[4:260].view(np.int8).astype(np.int32)
        bs = blk[260:292].view(np.int16)
        xb = x[256 * b:256 * (b + 1)]
        assert np.array_equal(bs, qs.reshape(16, 16).sum(1))
        assert qs.max() <= 127 and qs.min() >= -128
        assert np.max(np.abs(qs * dq - xb)) <= abs(dq) * 0.5 + 1e-6
    # block 0: max |x| = 5 at a negative value -> iscale = -127/-5 > 0, q = -127 there
    assert out[4 + 100].view(np.int8) == -127


def test_vec_dot_q4_K_matches_dequant_dot():
    rng = np.random.default_rng(11)
    K, N = 1024, 16
    w = helpers.rand_q4_K(rng, N, K)
    x = rng.standard_normal((3, K)).astype(np.float32)
    y = py_oracle.gemv(12, w, x, N)
    wd = py_oracle.dequant_q4_K(w, K, N).astype(np.float64)
    exact = x.astype(np.float64) @ wd.T
    # difference = activation quantization to Q8_K (<= half a step per element)
    bound = (np.abs(wd).sum(1)[None, :] * np.abs(x).max(1, keepdims=True) / 127.0) * 0.5 + 1e-5
    assert np.all(np.abs(y - exact) <= bound)


def test_vec_dot_q8_0_matches_dequant_dot():
    rng = np.random.default_rng(12)
    K, N = 2048, 8
    w = helpers.rand_q8_0(rng, N, K)
    x = rng.standard_normal((2, K)).astype(np.float32)
    y = py_oracle.gemv(8, w, x, N)
    wd = py_oracle.dequant_q8_0(w, K, N).astype(np.float64)
    exact = x.astype(np.float64) @ wd.T
    bound = (np.abs(wd).sum(1)[None, :] * np.abs(x).max(1, keepdims=True) / 127.0) * 0.51 + 1e-5
    assert np.all(np.abs(y - exact) <= bound)


def test_gelu_table_vs_formula():
    L = py_oracle.lib()
    golden = np.load(__import__("pathlib").Path(__file__).parent / "golden" / "ops_golden.npz")
    xs, ys = golden["gelu_x"], golden["gelu_y"]
    got = np.array([L.ref_gelu_table(float(v)) for v in xs], dtype=np.float32)
    # table output is fp16-rounded: within half an fp16 ulp of torch's tanh-GELU (+ input rounding)
    err = np.abs(got - ys)
    assert np.all(err <= 2e-3 * np.maximum(np.abs(ys), 1.0))
    f = np.array([L.ref_gelu_f32(float(v)) for v in xs], dtype=np.float32)
    assert np.max(np.abs(f - ys)) < 1e-5
