"""DAC runner on the CPU oracle (no GPU): the graph builds, allocates and decodes codec tokens to
PCM of the expected length; values are finite, not saturated and deterministic."""
import numpy as np

import py_oracle
import ttship


def test_dac_tiny_decodes_on_oracle():
    cfg = ttship.dac_config(latent_dim=64, decoder_dim=64, rates=[2, 2, 2, 2], n_layers=4, max_frames=16)
    codes = np.random.default_rng(3).integers(0, cfg.codebook_size, size=(5, cfg.n_codebooks))
    d = ttship.Dac(py_oracle.iface(4), cfg)
    try:
        a = d.decode(codes)
        b = d.decode(codes)
        assert d.hop == 16 and a.shape == (5 * 16,)
        assert d.last_graph_nodes() > 100
    finally:
        d.close()
    assert np.all(np.isfinite(a)) and np.array_equal(a, b)
    assert np.max(np.abs(a)) < 1.0 and np.std(a) > 0.05
