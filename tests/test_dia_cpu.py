"""Dia-1.6B runner on the CPU oracle: build_dia_graph (src/models/dia/model.cpp:705-720) with the
encoder step, cross K/V store, GQA repeat-interleave self KV store and cfg_scale as graph ops."""
import numpy as np

import py_oracle
import ttship

TINY = dict(n_encoder_layers=1, n_decoder_layers=2, encoder_hidden_size=64, decoder_hidden_size=128, encoder_attn_heads=4,
            decoder_attn_heads=4, decoder_query_heads=2, head_size=32, encoder_ffn_size=128, decoder_ffn_size=256,
            max_generation_size=64, max_encoder_context_length=32)


def run(n_steps=4):
    d = ttship.Dia(py_oracle.iface(4), ttship.dia_config(**TINY))
    try:
        text = np.frombuffer(b"\x01 hello there.", dtype=np.uint8).astype(np.int32)
        lg = [d.prefill(text, np.full(9, 1026, dtype=np.int32))]
        for _ in range(n_steps):
            lg.append(d.decode(lg[-1].argmax(axis=1).astype(np.int32)))
        assert d.position() == n_steps + 1
        st = d.plan_stats()
        return np.stack(lg), st
    finally:
        d.close()


def test_dia_tiny_deterministic_and_finite():
    a, st = run()
    b, _ = run()
    assert np.array_equal(a, b)
    assert np.isfinite(a).all() and a.shape == (5, 9, 1028)
    # per decoder layer: self-attention over the transposed V cache and cross-attention fused
    assert st["attn"] == 2 * TINY["n_decoder_layers"], st
    assert st["rint"] == 2 * TINY["n_decoder_layers"], st  # K and V repeat_interleave chains: one pass each


def test_dia_generate_matches_decode_loop():
    text = np.frombuffer(b"\x01 hi.", dtype=np.uint8).astype(np.int32)
    a = ttship.Dia(py_oracle.iface(4), ttship.dia_config(**TINY))
    b = ttship.Dia(py_oracle.iface(4), ttship.dia_config(**TINY))
    try:
        first = a.prefill(text, np.full(9, 1026, dtype=np.int32)).argmax(axis=1).astype(np.int32)
        b.prefill(text, np.full(9, 1026, dtype=np.int32))
        toks = a.generate(first, 5)
        audio = first
        for s in range(5):
            audio = b.decode(audio).argmax(axis=1).astype(np.int32)
            assert np.array_equal(audio, toks[s])
    finally:
        a.close()
        b.close()
