"""Weight quantizers on the CPU oracle (quantize_row_q4_K_ref / quantize_row_q8_0_ref restated in
oracle/ggml_ref.c): known answers, structural invariants of the blocks, and round-trip error bounds.
The HIP quantizer is compared byte for byte against these in tests/test_quant_gpu.py.

Parity with ggml's own quantizer binary is unpinned (the ggml submodule is absent); the restatement
follows ggml-quants.c's source order with every operation rounded to f32."""
import numpy as np
import pytest

import py_oracle
import ttship


def special_rows(K=512, seed=0):
    """Rows that hit the quantizer's branches: zeros, a constant, one sign only, a single spike,
    tiny and huge magnitudes, and Gaussian weights at two scales."""
    rng = np.random.default_rng(seed)
    rows = [np.zeros(K), np.full(K, 0.37), -np.abs(rng.standard_normal(K)), np.abs(rng.standard_normal(K)),
            np.where(np.arange(K) == 77, 5.0, 0.0), rng.standard_normal(K) * 1e-6, rng.standard_normal(K) * 300.0,
            rng.standard_normal(K) * 0.02, rng.standard_normal(K)]
    mixed = rng.standard_normal(K)
    mixed[:32] = 0.0  # one all-zero sub-block inside a live block
    rows.append(mixed)
    return np.asarray(rows, dtype=np.float32)


def q4k_fields(q, n):
    b = q.reshape(n, 144)
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32).reshape(-1)
    dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32).reshape(-1)
    return b, d, dmin


def scale_min(sc, j):
    """get_scale_min_k4"""
    if j < 4:
        return sc[j] & 63, sc[j + 4] & 63
    return (sc[j + 4] & 0xF) | ((sc[j - 4] >> 6) << 4), (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4)


def test_q4_K_blocks_and_round_trip():
    x = special_rows()
    N, K = x.shape
    q = py_oracle.quantize(ttship.Q4_K, x)
    assert q.shape == (N * K // 256 * 144,)
    b, d, dmin = q4k_fields(q, N * K // 256)
    assert np.all(d >= 0) and np.all(dmin >= 0)
    # row 0 (zeros) quantizes to an all-zero block
    assert not b[0:2].any()
    y = py_oracle.dequant_q4_K(q, K, N)
    for r in range(N):
        for blk in range(K // 256):
            i = r * (K // 256) + blk
            for j in range(8):
                sl = slice(256 * blk + 32 * j, 256 * blk + 32 * (j + 1))
                sc, mn = scale_min(b[i, 4:16], j)
                assert sc <= 63 and mn <= 63
                # codes reproduce the values to within one code step of the sub-block (the weighted
                # search may trade the extremes), and the sub-block's range is covered
                step = float(d[i]) * sc
                err = float(np.max(np.abs(y[r, sl] - x[r, sl])))
                # row 5 (|x| ~ 1e-6): d = max_scale / 63 is an fp16 subnormal (or 0), whose coarse
                # steps bound the error by a few |x| instead
                amax = float(np.max(np.abs(x[r, sl])))
                tol = 2.5 * amax if d[i] < 6.1e-5 else 1e-6 * max(1.0, amax)
                assert err <= step + tol, (r, blk, j, err, step)
    # Gaussian rows: relative RMS error of a 4.5-bit format
    for r in (7, 8):
        rel = np.sqrt(np.mean((y[r] - x[r]) ** 2) / np.mean(x[r] ** 2))
        assert rel < 0.12, rel


def test_q4_K_constant_and_spike_are_near_exact():
    x = special_rows()
    y = py_oracle.dequant_q4_K(py_oracle.quantize(ttship.Q4_K, x), x.shape[1], x.shape[0])
    assert np.max(np.abs(y[1] - 0.37)) < 0.37 / 15  # constant row
    assert abs(y[4][77] - 5.0) < 5.0 / 15 and np.max(np.abs(np.delete(y[4], 77))) < 5.0 / 15


def test_q4_K_deterministic_and_row_independent():
    x = special_rows(seed=3)
    a = py_oracle.quantize(ttship.Q4_K, x)
    b = py_oracle.quantize(ttship.Q4_K, x)
    assert np.array_equal(a, b)
    rs = x.shape[1] // 256 * 144
    one = py_oracle.quantize(ttship.Q4_K, x[5:6])
    assert np.array_equal(one, a[5 * rs:6 * rs])


def test_q8_0_known_answer():
    x = np.zeros((1, 64), np.float32)
    x[0, :32] = np.arange(-16, 16) * 2.0
    x[0, 5] = 127.0
    x[0, 32:] = 0.5
    q = py_oracle.quantize(ttship.Q8_0, x).reshape(2, 34)
    d0 = q[0, :2].copy().view(np.float16)[0]
    assert d0 == np.float16(1.0)
    qs = q[0, 2:].view(np.int8)
    ref = np.round(x[0, :32]).astype(np.int8)  # d = 127 / 127 = 1
    assert np.array_equal(qs, ref)
    d1 = float(q[1, :2].copy().view(np.float16)[0])
    assert d1 == pytest.approx(0.5 / 127, rel=1e-3) and np.all(q[1, 2:].view(np.int8) == 127)
