"""DAC decoder (codec tokens -> PCM) end to end: HIP backend vs the CPU oracle on the same graph
and the same synthetic weights.  Bar (north_star): PCM samples within 1e-4 absolute."""
import numpy as np
import pytest

import py_oracle
import ttship

CFGS = {
    "tiny": dict(latent_dim=64, decoder_dim=64, rates=[2, 2, 2, 2], n_layers=4, max_frames=16),
    "dac44k_narrow": dict(latent_dim=256, decoder_dim=384, rates=[8, 8, 4, 2], n_layers=4, max_frames=8),
}


def decode(iface, cfg, codes):
    d = ttship.Dac(iface, cfg)
    try:
        return d.decode(codes)
    finally:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,T", [("tiny", 6), ("dac44k_narrow", 4)])
def test_dac_pcm_matches_oracle(hip, name, T):
    cfg = ttship.dac_config(**CFGS[name])
    codes = np.random.default_rng(11).integers(0, cfg.codebook_size, size=(T, cfg.n_codebooks))
    gpu = decode(hip.iface(), cfg, codes)
    ref = decode(py_oracle.iface(8), cfg, codes)
    assert gpu.shape == ref.shape == (T * int(np.prod(CFGS[name]["rates"])),)
    assert np.all(np.isfinite(gpu))
    err = float(np.max(np.abs(gpu.astype(np.float64) - ref)))
    assert err <= 1e-4, f"max |pcm_gpu - pcm_oracle| = {err:.3e}"
    assert float(np.std(ref)) > 0.05  # not a degenerate (saturated / silent) decoder
