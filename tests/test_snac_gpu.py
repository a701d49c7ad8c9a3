"""SNAC decoder (Orpheus' vocoder: three codebook streams -> 24 kHz PCM) end to end: HIP backend vs
the CPU oracle on the same graph, synthetic weights and noise draws.  Bar (north_star): PCM
samples within 1e-4 absolute."""
import numpy as np
import pytest

import py_oracle
import ttship

CFGS = {
    "tiny": dict(latent_dim=32, decoder_dim=64, codebook_size=64, rates=[2, 2, 4, 2], max_frames=32),
    "snac24k": dict(max_frames=16),
}


def decode(iface, cfg, heads, noise):
    s = ttship.Snac(iface, cfg)
    try:
        return s.decode(heads, noise), s.last_graph_nodes()
    finally:
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,T", [("tiny", 12), ("snac24k", 8), ("snac24k", 16)])
def test_snac_pcm_matches_oracle(hip, name, T):
    cfg = ttship.snac_config(**CFGS[name])
    rng = np.random.default_rng(5 + T)
    heads = [rng.integers(0, cfg.codebook_size, size=T // cfg.repeats[i]) for i in range(cfg.n_heads)]
    npf = sum(int(np.prod(list(cfg.rates)[:l + 1])) for l in range(cfg.n_layers))
    noise = rng.standard_normal(npf * T).astype(np.float32)
    gpu, nodes = decode(hip.iface(), cfg, heads, noise)
    ref, _ = decode(py_oracle.iface(8), cfg, heads, noise)
    hop = int(np.prod(list(cfg.rates)[:cfg.n_layers]))
    assert gpu.shape == ref.shape == (T * hop,)
    assert np.all(np.isfinite(gpu))
    err = float(np.max(np.abs(gpu.astype(np.float64) - ref)))
    print(f"snac {name} T {T} nodes {nodes} max err {err:.3e}")
    assert err <= 1e-4, f"max |pcm_gpu - pcm_oracle| = {err:.3e}"
    assert float(np.std(ref)) > 1e-2  # not a degenerate (saturated / silent) decoder
