"""DAC runner on the CPU oracle (no GPU): the graph builds, allocates and decodes codec tokens to
PCM of the expected length; values are finite, not saturated and deterministic."""
import numpy as np
import pytest

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


def _batch_vs_single(iface, cfg, nb, T, gap, seed):
    codes = np.random.default_rng(seed).integers(0, cfg.codebook_size, size=(nb, T, cfg.n_codebooks))
    d = ttship.Dac(iface, cfg)
    try:
        single = np.stack([d.decode(codes[z]) for z in range(nb)])
        batched = d.decode_batch(codes, gap=gap)
        g = d.min_gap
    finally:
        d.close()
    return single, batched, g


def test_dac_batch_bit_identical_on_oracle():
    """tts_dac_decode_batch: nb prompts laid out along time with zeroed gaps, one graph, on the oracle
    (the reference ops' semantics): every prompt's PCM equals its own decode bit for bit."""
    cfg = ttship.dac_config(latent_dim=64, decoder_dim=64, rates=[8, 8, 4, 2], n_layers=4, max_frames=64)
    single, batched, g = _batch_vs_single(py_oracle.iface(8), cfg, 3, 5, 0, 11)
    assert g == 4  # the k 7, dilation 9 convs reach 27 samples at rate 8
    assert np.array_equal(single, batched)


def test_dac_batch_slow_rates_and_wider_gap():
    cfg = ttship.dac_config(latent_dim=64, decoder_dim=64, rates=[2, 2, 2, 2], n_layers=4, max_frames=96)
    single, batched, g = _batch_vs_single(py_oracle.iface(8), cfg, 4, 3, 20, 12)
    assert g == 14  # 27 samples at rate 2
    assert np.array_equal(single, batched)


def test_dac_batch_rejects_short_gap_and_overflow():
    cfg = ttship.dac_config(latent_dim=64, decoder_dim=64, rates=[8, 8, 4, 2], n_layers=4, max_frames=16)
    d = ttship.Dac(py_oracle.iface(4), cfg)
    try:
        codes = np.zeros((2, 4, cfg.n_codebooks), np.int32)
        with pytest.raises(RuntimeError):
            d.decode_batch(codes, gap=3)  # below the minimum gap of 4
        with pytest.raises(RuntimeError):
            d.decode_batch(np.zeros((4, 4, cfg.n_codebooks), np.int32))  # 4 * 4 + 3 * 4 > 16 frames
        assert d.decode_batch(codes[:1]).shape == (1, 4 * d.hop)  # nb = 1: the plain decode
    finally:
        d.close()


def test_dac_batch_rejects_odd_rates():
    """An odd upsampling rate s has padding ceil(s / 2): a transposed conv then outputs T s - 1 samples,
    which the batched layout (prompt z at z * (T + gap) * hop) cannot hold -- refused; the
    single decode still works."""
    cfg = ttship.dac_config(latent_dim=64, decoder_dim=64, rates=[8, 5, 4, 3], n_layers=4, max_frames=64)
    d = ttship.Dac(py_oracle.iface(4), cfg)
    try:
        codes = np.zeros((2, 4, cfg.n_codebooks), np.int32)
        with pytest.raises(RuntimeError):
            d.decode_batch(codes)
        assert np.all(np.isfinite(d.decode(codes[0])))
    finally:
        d.close()


def test_dac_batch_masks_fused_into_snakes():
    """The batched graph's gap masks ride in the snake passes (k_snake's mask operand): the same items
    as a single decode plus the one mask product in front of the first conv."""
    cfg = ttship.dac_config(latent_dim=64, decoder_dim=64, rates=[8, 8, 4, 2], n_layers=4, max_frames=64)
    d = ttship.Dac(py_oracle.iface(4), cfg)
    try:
        codes = np.zeros((3, 4, cfg.n_codebooks), np.int32)
        d.decode(codes[0])
        one = d.plan_stats()
        d.decode_batch(codes)
        many = d.plan_stats()
    finally:
        d.close()
    assert one["snake"] == many["snake"] == 4 * 7 + 1
    assert many["unfused"] == one["unfused"] + 1, (one, many)
