"""The oracle's SIMD accumulation mode (oracle_set_simd_mode(1), oracle/ggml_ref.c): the x86
AVX2 / FMA / F16C order of ggml-cpu's vec_dot_f16 / _f32 / q4_K_q8_K / q8_0_q8_0.  Each restatement is
checked bit for bit against an independent exact-arithmetic emulation of the lane structure (Fractions,
correctly rounded to f32), and against the scalar mode within a few ulps.  scripts/simd_gap.py uses the
mode to measure how far the two CPU orders themselves drift apart on the models."""
import ctypes
from fractions import Fraction

import numpy as np

import py_oracle
import ttship


def f32(fr):
    """Fraction -> nearest float32, ties to even (exact: no double rounding)."""
    c = np.float32(float(fr))
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        if not np.isfinite(cand):
            continue
        d = abs(Fraction(float(cand)) - fr)
        if best is None or d < best[0] or (d == best[0] and (int(cand.view(np.uint32)) & 1) == 0):
            best = (d, cand)
    return best[1]


def fma(a, b, c):
    return f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def add(a, b):
    return f32(Fraction(float(a)) + Fraction(float(b)))


def reduce4x8(acc):
    acc = [list(a) for a in acc]
    for e in range(8):
        acc[0][e] = add(acc[0][e], acc[2][e])
        acc[1][e] = add(acc[1][e], acc[3][e])
    for e in range(8):
        acc[0][e] = add(acc[0][e], acc[1][e])
    t0 = [add(acc[0][e], acc[0][4 + e]) for e in range(4)]
    return add(add(t0[0], t0[1]), add(t0[2], t0[3]))


def hsum8(x):
    r = [add(x[4 + e], x[e]) for e in range(4)]
    return add(add(r[0], r[2]), add(r[1], r[3]))


def emu_dot_f32(x, y):
    n = len(x)
    np_ = n & ~31
    acc = [[np.float32(0)] * 8 for _ in range(4)]
    for i in range(0, np_, 32):
        for j in range(4):
            for e in range(8):
                acc[j][e] = fma(x[i + 8 * j + e], y[i + 8 * j + e], acc[j][e])
    s = reduce4x8(acc)
    for i in range(np_, n):
        s = fma(x[i], y[i], s)
    return s


def emu_dot_f16(xh, yh):
    x, y = xh.astype(np.float32), yh.astype(np.float32)
    n = len(x)
    np_ = n & ~31
    acc = [[np.float32(0)] * 8 for _ in range(4)]
    for i in range(0, np_, 32):
        for j in range(4):
            for e in range(8):
                acc[j][e] = fma(x[i + 8 * j + e], y[i + 8 * j + e], acc[j][e])
    s = float(reduce4x8(acc))
    for i in range(np_, n):
        s += float(x[i]) * float(y[i])  # ggml_float tail
    return np.float32(s)


def call_dot(name, n, x, y):
    out = ctypes.c_float()
    getattr(py_oracle.lib(), name)(n, ctypes.byref(out), x.ctypes.data, y.ctypes.data)
    return np.float32(out.value)


def test_simd_dot_f32_f16_bit_exact_vs_emulation():
    rng = np.random.default_rng(4)
    for n in (32, 64, 100, 257):
        x = rng.standard_normal(n).astype(np.float32)
        y = rng.standard_normal(n).astype(np.float32)
        with py_oracle.simd_mode(1):
            got = call_dot("ref_vec_dot_f32", n, x, y)
        assert got == emu_dot_f32(x, y), n
        xh, yh = x.astype(np.float16), y.astype(np.float16)
        with py_oracle.simd_mode(1):
            got16 = call_dot("ref_vec_dot_f16", n, xh, yh)
        assert got16 == emu_dot_f16(xh, yh), n
        with py_oracle.simd_mode(0):
            ref = call_dot("ref_vec_dot_f32", n, x, y)
        assert abs(float(got) - float(ref)) <= 1e-5 * float(np.sum(np.abs(x * y)))


def q4k_emu(wb, xq, K):
    """ggml_vec_dot_q4_K_q8_K (__AVX2__) over one row: lanes of 4 bytes per 32-byte chunk."""
    w = np.frombuffer(wb, dtype=np.uint8)
    q = np.frombuffer(xq, dtype=np.uint8)
    acc = [np.float32(0)] * 8
    acc_m = [np.float32(0)] * 4
    for i in range(K // 256):
        blk = w[i * 144:(i + 1) * 144]
        yb = q[i * 292:(i + 1) * 292]
        yd = yb[:4].view(np.float32)[0]
        yq = yb[4:260].view(np.int8).astype(np.int64)
        bsums = yb[260:292].view(np.int16).astype(np.int64)
        xd = blk[0:2].view(np.float16)[0].astype(np.float32)
        xdmin = blk[2:4].view(np.float16)[0].astype(np.float32)
        sc12 = blk[4:16]
        qs = blk[16:144]
        sc, mn = [], []
        for j in range(8):  # get_scale_min_k4
            if j < 4:
                sc.append(int(sc12[j]) & 63)
                mn.append(int(sc12[j + 4]) & 63)
            else:
                sc.append((int(sc12[j + 4]) & 0xF) | ((int(sc12[j - 4]) >> 6) << 4))
                mn.append((int(sc12[j + 4]) >> 4) | ((int(sc12[j]) >> 6) << 4))
        d = np.float32(yd * xd)
        dmin = np.float32(-yd * xdmin)
        for qi in range(4):
            s0 = bsums[4 * qi] + bsums[4 * qi + 1]
            s1 = bsums[4 * qi + 2] + bsums[4 * qi + 3]
            acc_m[qi] = fma(dmin, np.float32(mn[2 * qi] * s0 + mn[2 * qi + 1] * s1), acc_m[qi])
        sumi = [0] * 8
        for j in range(4):
            chunk = qs[32 * j:32 * j + 32].astype(np.int64)
            lo8, hi8 = yq[64 * j:64 * j + 32], yq[64 * j + 32:64 * j + 64]
            for k in range(8):
                b = slice(4 * k, 4 * k + 4)
                sumi[k] += sc[2 * j] * int(np.sum((chunk[b] & 0xF) * lo8[b])) + sc[2 * j + 1] * int(np.sum((chunk[b] >> 4) * hi8[b]))
        for k in range(8):
            acc[k] = fma(d, np.float32(sumi[k]), acc[k])
    return add(hsum8(acc), add(add(acc_m[0], acc_m[2]), add(acc_m[1], acc_m[3])))


def q80_emu(wb, xq, K):
    w = np.frombuffer(wb, dtype=np.uint8)
    q = np.frombuffer(xq, dtype=np.uint8)
    acc = [np.float32(0)] * 8
    for ib in range(K // 32):
        xb, yb = w[ib * 34:(ib + 1) * 34], q[ib * 34:(ib + 1) * 34]
        d = np.float32(xb[:2].view(np.float16)[0].astype(np.float32) * yb[:2].view(np.float16)[0].astype(np.float32))
        xs, ys = xb[2:].view(np.int8).astype(np.int64), yb[2:].view(np.int8).astype(np.int64)
        for k in range(8):
            acc[k] = fma(d, np.float32(int(np.sum(xs[4 * k:4 * k + 4] * ys[4 * k:4 * k + 4]))), acc[k])
    return hsum8(acc)


def test_simd_dot_quantized_bit_exact_vs_emulation():
    rng = np.random.default_rng(6)
    L = py_oracle.lib()
    K = 512
    for wtype, emu, act_bytes, quant_act in ((ttship.Q4_K, q4k_emu, 292, L.ref_quantize_row_q8_K),
                                             (ttship.Q8_0, q80_emu, 34, L.ref_quantize_row_q8_0)):
        blk = 256 if wtype == ttship.Q4_K else 32
        for row in range(3):
            w = (rng.standard_normal((1, K)) * (0.02 if row else 3.0)).astype(np.float32)
            x = rng.standard_normal(K).astype(np.float32)
            wb = py_oracle.quantize(wtype, w)
            xq = np.zeros(K // blk * act_bytes, dtype=np.uint8)
            quant_act(x.ctypes.data, xq.ctypes.data, K)
            fn = "ref_vec_dot_q4_K_q8_K" if wtype == ttship.Q4_K else "ref_vec_dot_q8_0_q8_0"
            with py_oracle.simd_mode(1):
                got = call_dot(fn, K, wb, xq)
            assert got == emu(wb.tobytes(), xq.tobytes(), K), (wtype, row)
            with py_oracle.simd_mode(0):
                ref = call_dot(fn, K, wb, xq)
            assert abs(float(got) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))


def test_simd_mode_gemv_drift_is_ulps():
    """Through the threaded GEMV path: every output within a few ulps of the scalar order."""
    rng = np.random.default_rng(0)
    K, N, M = 1024, 128, 3
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    x = rng.standard_normal((M, K)).astype(np.float32)
    for t in (ttship.Q4_K, ttship.Q8_0, ttship.F16, ttship.F32):
        wb = (py_oracle.quantize(t, w) if t in (ttship.Q4_K, ttship.Q8_0)
              else w.astype(np.float16).view(np.uint8).ravel() if t == ttship.F16 else w.view(np.uint8).ravel())
        with py_oracle.simd_mode(0):
            a = py_oracle.gemv(t, wb, x, N)
        with py_oracle.simd_mode(1):
            b = py_oracle.gemv(t, wb, x, N)
        assert np.max(np.abs(a - b)) <= 1e-6 * np.max(np.abs(a)), t
        assert np.mean(a != b) > 0.3, t  # and the order really differs
    assert py_oracle.lib().oracle_simd_mode() == 0
