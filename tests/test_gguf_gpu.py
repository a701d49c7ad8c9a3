"""The GGUF path on the device: the quantize tool with the device quantizers (tts_hip_gguf_quantize)
writes the same file bytes as with the CPU oracle's quantize_row_q4_K_ref / _q8_0_ref, and runners
loaded from a quantized file (runner_from_file -> assign_weight) on the HIP backend decode exactly like
the oracle loaded from the same file: greedy tokens bit-exact, logits within 1e-4, DAC PCM identical."""
import numpy as np
import pytest

import py_oracle
import ttship
from test_gguf_cpu import DAC_TINY, TINY, _oracle_rows


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("gguf_gpu")
    cfg32 = ttship.parler_config(weight_type=ttship.F32, head_type=ttship.F32, **TINY)
    src = d / "parler-f32.gguf"
    ttship.write_parler_synthetic_gguf(src, cfg32, ttship.dac_config(**DAC_TINY))
    return d, src


@pytest.mark.gpu
@pytest.mark.parametrize("qtype", [ttship.Q4_K, ttship.Q8_0])
def test_device_quantize_tool_bytes(hip, files, qtype):
    d, src = files
    dev, ref = d / f"dev-{qtype}.gguf", d / f"ref-{qtype}.gguf"
    p = ttship.quantize_params(qtype, quantize_output_heads=1)
    ttship.quantize_gguf(src, dev, p, backend=hip)
    ttship.quantize_gguf(src, ref, p, rows_fn=_oracle_rows)
    assert dev.read_bytes() == ref.read_bytes()


@pytest.mark.gpu
def test_parler_from_quantized_gguf_matches_oracle(hip, files):
    d, src = files
    q4 = d / "parler-q4_k-dev.gguf"
    ttship.quantize_gguf(src, q4, ttship.quantize_params(ttship.Q4_K), backend=hip)
    with ttship.Gguf(q4) as g:
        cfg = ttship.parler_config_from_gguf(g, max_ctx=TINY["max_ctx"], batch=2)
        dev = ttship.Parler(hip.iface(), cfg, gguf=g)
        ref = ttship.Parler(py_oracle.iface(8), cfg, gguf=g)
    try:
        prompt = (np.arange(10, dtype=np.int32).reshape(2, 5) * 53) % TINY["prompt_vocab"]
        for r in (dev, ref):
            r.prefill(prompt)
        la = dev.decode(np.full((2, 9), 1025, dtype=np.int32))
        lb = ref.decode(np.full((2, 9), 1025, dtype=np.int32))
        assert np.max(np.abs(la - lb)) <= 1e-4
        ta, tb = dev.generate(12), ref.generate(12)
        assert np.array_equal(ta, tb)
    finally:
        dev.close()
        ref.close()


@pytest.mark.gpu
def test_dac_from_gguf_matches_oracle(hip, files):
    _, src = files
    codes = np.random.default_rng(9).integers(0, 1024, size=(6, 9))
    with ttship.Gguf(src) as g:
        cfg = ttship.dac_config_from_gguf(g, max_frames=DAC_TINY["max_frames"])
        dev = ttship.Dac(hip.iface(), cfg, gguf=g)
        ref = ttship.Dac(py_oracle.iface(8), cfg, gguf=g)
    try:
        assert np.array_equal(dev.decode(codes), ref.decode(codes))
    finally:
        dev.close()
        ref.close()
