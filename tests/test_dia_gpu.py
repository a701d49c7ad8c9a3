"""Dia-1.6B parity: HIP backend vs CPU oracle on the same graphs (build_dia_graph,
src/models/dia/model.cpp:705-720): encoder step + cross K/V store, then CFG decoder steps.

Bars: greedy heads' argmax identical every step; logits within 1e-4 * max|logit| + 1e-4."""
import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_encoder_layers=1, n_decoder_layers=2, encoder_hidden_size=64, decoder_hidden_size=128, encoder_attn_heads=4,
            decoder_attn_heads=4, decoder_query_heads=2, head_size=32, encoder_ffn_size=128, decoder_ffn_size=256,
            max_generation_size=64, max_encoder_context_length=32)
# real Dia widths (2048 / 16 x 128 / 4 KV groups / 8192, encoder 1024 over 1024 positions), fewer layers
WIDE = dict(n_encoder_layers=1, n_decoder_layers=2, max_generation_size=32)


def run_pair(hip, kw, steps):
    g = ttship.Dia(hip.iface(), ttship.dia_config(**kw))
    c = ttship.Dia(py_oracle.iface(16), ttship.dia_config(**kw))
    try:
        text = np.frombuffer(b"\x01 The birch canoe slid on the smooth planks. \x02 Glue the sheet.", dtype=np.uint8).astype(np.int32)
        text = text[: c.cfg.max_encoder_context_length]
        audio = np.full(9, 1026, dtype=np.int32)
        for s in range(steps + 1):
            lg = g.prefill(text, audio) if s == 0 else g.decode(audio)
            lc = c.prefill(text, audio) if s == 0 else c.decode(audio)
            tol = 1e-4 * np.abs(lc).max() + 1e-4
            assert np.abs(lg - lc).max() <= tol, (s, np.abs(lg - lc).max())
            assert np.array_equal(lg.argmax(axis=1), lc.argmax(axis=1)), s
            audio = lc.argmax(axis=1).astype(np.int32)
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_dia_tiny(hip):
    run_pair(hip, TINY, 8)


@pytest.mark.gpu
def test_dia_wide_two_layers(hip):
    run_pair(hip, WIDE, 3)


@pytest.mark.gpu
def test_dia_generate_device_loop(hip):
    """The device-resident greedy loop (plans + greedy_step) gives the oracle's host-loop tokens."""
    g = ttship.Dia(hip.iface(), ttship.dia_config(**TINY))
    c = ttship.Dia(py_oracle.iface(16), ttship.dia_config(**TINY))
    try:
        text = np.frombuffer(b"\x01 It's easy to tell the depth.", dtype=np.uint8).astype(np.int32)[:32]
        first = c.prefill(text, np.full(9, 1026, dtype=np.int32)).argmax(axis=1).astype(np.int32)
        assert np.array_equal(g.prefill(text, np.full(9, 1026, dtype=np.int32)).argmax(axis=1), first)
        tg, tc = g.generate(first, 12), c.generate(first, 12)
        assert np.array_equal(tg, tc), f"{tg}\n{tc}"
        assert g.position() == c.position() == 13
    finally:
        g.close()
        c.close()
