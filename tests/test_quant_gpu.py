"""Device weight quantizers (tts_hip_quantize, k_quant.hip) vs the CPU oracle's
quantize_row_q4_K_ref / quantize_row_q8_0_ref: identical bytes over the quantizer's branch cases and
over Parler / Orpheus-shaped Gaussian matrices; a GEMV on the device-quantized matrix then equals the
oracle's GEMV on the oracle-quantized one."""
import numpy as np
import pytest

import py_oracle
import ttship
from test_quant_cpu import special_rows


@pytest.mark.gpu
@pytest.mark.parametrize("wtype", [ttship.Q4_K, ttship.Q8_0])
def test_quantize_special_rows_bytes(hip, wtype):
    x = special_rows(K=1024, seed=7)
    got = hip.quantize(wtype, x)
    ref = py_oracle.quantize(wtype, x)
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


@pytest.mark.gpu
@pytest.mark.parametrize("wtype,N,K,std", [(ttship.Q4_K, 1024, 1024, 0.02), (ttship.Q4_K, 300, 4096, 1.0),
                                           (ttship.Q4_K, 64, 3072, 0.05), (ttship.Q8_0, 512, 2048, 0.02)])
def test_quantize_matrix_bytes_and_gemv(hip, wtype, N, K, std):
    rng = np.random.default_rng(N + K)
    w = (rng.standard_normal((N, K)) * std).astype(np.float32)
    got = hip.quantize(wtype, w)
    ref = py_oracle.quantize(wtype, w)
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, f"{bad.size} of {ref.size} bytes differ"
    x = rng.standard_normal((3, K)).astype(np.float32)
    y = py_oracle.gemv(wtype, got, x, N)
    yr = py_oracle.gemv(wtype, ref, x, N)
    assert np.array_equal(y, yr)
