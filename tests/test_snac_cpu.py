"""SNAC decoder runner (Orpheus' vocoder) on the CPU oracle (no GPU), checked against an
independent float32 PyTorch restatement of the published SNAC decoder (tests/snac_ref.py).

Two bars: (1) against the restatement with the oracle's arithmetic (conv inputs and kernels
rounded to f16 as ggml's im2col / vec_dot_type do, exact products summed in f64, correctly rounded
sin): every named intermediate bit-identical, PCM within 1 ulp of tanh; (2) against plain fp32
PyTorch (the model's own semantics), PCM within 1e-2 of its peak: torch's f32 sin and
accumulations differ in the last bit, and ~20 convs that re-round their inputs to f16 amplify that
to f16-level steps."""
import numpy as np
import pytest

import py_oracle
import snac_ref
import ttship

TINY = dict(latent_dim=32, decoder_dim=64, codebook_size=64, rates=[2, 2, 4, 2], max_frames=32)


def codes_and_noise(cfg, T, seed, npf):
    rng = np.random.default_rng(seed)
    heads = [rng.integers(0, cfg.codebook_size, size=T // cfg.repeats[i]) for i in range(cfg.n_heads)]
    noise = rng.standard_normal(npf * T).astype(np.float32)
    return heads, noise


@pytest.mark.parametrize("T,seed", [(4, 0), (12, 1)])
def test_snac_oracle_matches_torch(T, seed):
    cfg = ttship.snac_config(**TINY, debug_no_reuse=1, arena_bytes=128 << 20)
    s = ttship.Snac(py_oracle.iface(8), cfg)
    try:
        assert s.hop == 32 and s.noise_per_frame == 2 + 4 + 16 + 32
        heads, noise = codes_and_noise(cfg, T, seed, s.noise_per_frame)
        pcm = s.decode(heads, noise)
        W = s.weights()
        taps = {}
        ref16 = snac_ref.decode(cfg, W, heads, noise, f16=True, taps=taps)
        ref = snac_ref.decode(cfg, W, heads, noise)
        assert pcm.shape == ref.shape == ref16.shape == (T * s.hop,)
        assert np.all(np.isfinite(pcm))
        assert len(taps) == 3 + 4 * 5
        for name, v in taps.items():
            got = s.node(name)
            assert got is not None and np.array_equal(got, v.numpy().reshape(-1)), name
        err16 = float(np.max(np.abs(pcm - ref16)))
        assert err16 <= 1.2e-7, err16
        err = float(np.max(np.abs(pcm - ref)))
        assert err <= 1e-2 * float(np.max(np.abs(ref))), err
        assert float(np.std(pcm)) > 1e-2 and float(np.max(np.abs(pcm))) < 1.0
        assert s.last_graph_nodes() > 150
    finally:
        s.close()


def test_snac_deterministic_and_rejects_ragged_heads():
    cfg = ttship.snac_config(**TINY)
    s = ttship.Snac(py_oracle.iface(4), cfg)
    try:
        heads, noise = codes_and_noise(cfg, 8, 3, s.noise_per_frame)
        assert np.array_equal(s.decode(heads, noise), s.decode(heads, noise))
        with pytest.raises(ValueError):
            s.decode(heads, noise[:-1])
        bad = [h[:1] for h in heads[:2]] + [heads[2][:6]]  # T = 6 is not a multiple of the coarsest stride 4
        with pytest.raises(RuntimeError):
            s.decode(bad, np.zeros(6 * s.noise_per_frame, np.float32))
    finally:
        s.close()
