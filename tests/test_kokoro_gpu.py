"""Kokoro iSTFTNet generator end to end: HIP backend vs the CPU oracle on the same graph, the same
synthetic weights and the same host-side uv / noise / envelope inputs.  Bar (north_star): PCM
samples within 1e-4 absolute.  The oracle itself is checked against a PyTorch restatement of
Kokoro's generator in tests/test_kokoro_cpu.py."""
import numpy as np
import pytest

import py_oracle
import ttship
from test_kokoro_cpu import inputs

CFGS = {
    "tiny": dict(in_channels=32, style_dim=16, max_frames=16),
    "narrow": dict(in_channels=128, style_dim=64, max_frames=16),
    "kokoro82m": dict(max_frames=8),
}


def run(iface, cfg, args):
    k = ttship.KokoroGenerator(iface, cfg)
    try:
        return k.run(*args)
    finally:
        k.close()


@pytest.mark.gpu
@pytest.mark.parametrize("acc", [0, 2])  # TTS_HIP_OPT_CONV_F32ACC (see test_dac_gpu.py)
@pytest.mark.parametrize("name,T,seed", [("tiny", 4, 0), ("tiny", 7, 1), ("narrow", 9, 2), ("kokoro82m", 4, 3)])
def test_kokoro_generator_pcm_matches_oracle(hip, name, T, seed, acc):
    cfg = ttship.kokoro_gen_config(**CFGS[name])
    args = inputs(cfg, T, seed)
    hip.set_option(ttship.OPT["CONV_F32ACC"], acc)
    try:
        gpu = run(hip.iface(), cfg, args)
    finally:
        hip.set_option(ttship.OPT["CONV_F32ACC"], 0)
    ref = run(py_oracle.iface(8), cfg, args)
    assert gpu.shape == ref.shape == (300 * T,)
    assert np.all(np.isfinite(gpu))
    err = float(np.max(np.abs(gpu.astype(np.float64) - ref)))
    print(f"kokoro {name} acc {acc} max err {err:.3e}")
    assert err <= (1e-4 if acc == 0 else 1e-3), f"max |pcm_gpu - pcm_oracle| = {err:.3e}"  # mode 2: see test_dac_gpu.py
    assert float(np.std(ref)) > 1e-2


@pytest.mark.gpu
def test_kokoro_generator_all_unvoiced_and_repeat(hip):
    cfg = ttship.kokoro_gen_config(**CFGS["tiny"])
    args = inputs(cfg, 5, 4, f0=np.zeros(5))
    k = ttship.KokoroGenerator(hip.iface(), cfg)
    try:
        a = k.run(*args)
        b = k.run(*args)
    finally:
        k.close()
    ref = run(py_oracle.iface(8), cfg, args)
    assert np.array_equal(a, b)
    assert float(np.max(np.abs(a.astype(np.float64) - ref))) <= 1e-4
