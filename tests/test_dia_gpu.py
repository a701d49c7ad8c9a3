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


HARVARD = [b"The birch canoe slid on the smooth planks.", b"Glue the sheet to the dark blue background.",
           b"It's easy to tell the depth of a well.", b"These days a chicken leg is a rare dish.",
           b"Rice is often served in round bowls.", b"The juice of lemons makes fine punch.",
           b"The box was thrown beside the parked truck.", b"The hogs were fed chopped corn and garbage.",
           b"Four hours of steady work faced us.", b"A large size in stockings is hard to sell.",
           b"The boy was there when the sun rose.", b"A rod is used to catch pink salmon.",
           b"The source of the huge river is the clear spring.", b"Kick the ball straight and follow through.",
           b"Help the woman get back to her feet.", b"A pot of tea helps to pass the evening.",
           b"Smoky fires lack flame and heat.", b"The soft cushion broke the man's fall.",
           b"The salt breeze came across from the sea.", b"The girl at the booth sold fifty bonds.",
           b"The small pup gnawed a hole in the sock.", b"The fish twisted and turned on the bent hook.",
           b"Press the pants and sew a button on the vest.", b"The swan dive was far short of perfect.",
           b"The beauty of the view stunned the young boy.", b"Two blue fish swam in the tank."]


def dialogue(n_chars):
    """A two-speaker dialogue (Dia's [S1] / [S2] speaker tags as the tokenizer's bytes 0x01 / 0x02)
    of Harvard sentences, cut to n_chars bytes."""
    out, i = b"", 0
    while len(out) < n_chars:
        out += (b"\x01 " if i % 2 == 0 else b" \x02 ") + HARVARD[i % len(HARVARD)]
        i += 1
    return np.frombuffer(out[:n_chars], dtype=np.uint8).astype(np.int32)


def run_pair(hip, kw, steps, text=None):
    g = ttship.Dia(hip.iface(), ttship.dia_config(**kw))
    c = ttship.Dia(py_oracle.iface(16), ttship.dia_config(**kw))
    try:
        if text is None:
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


@pytest.mark.gpu
def test_dia_full_depth_long_dialogue(hip):
    """BASELINE configs[3] as configured: Dia-1.6B at full depth (18 decoder / 12 encoder layers,
    src/models/dia/model.h:65-85) over a long two-speaker dialogue near the 1024-byte encoder cap
    (model.cpp:668-670), 64 CFG decoder steps: argmax identical and logits within the bar every step."""
    text = dialogue(1000)
    assert len(text) == 1000
    run_pair(hip, dict(max_generation_size=80), 64, text=text)


@pytest.mark.gpu
def test_dia_q80_paths_bit_identical(hip):
    """Dia's decode GEMVs (Q8_0, 2 CFG columns) on every Q8_0 path: the (row, block)-per-thread kernel
    after separate norm + quantize launches with every graph fusion off (the reference point: one
    launch per node), the slab kernel after them, and the
    slab kernel quantizing -- after the RMS norms, normalizing -- the activation inside every workgroup
    (TTS_HIP_OPT_GEMV_Q80_PRO / _SLAB, the defaults), with the MLP's SILU * up folded into the up
    product's epilogue (TTS_FUSE_EPI) or not.  Same arithmetic, so every logit is bit-identical.  The
    prefill step runs the encoder's many-column Q8_0 GEMMs (the same epilogue at M = 2 x 32)."""
    text = np.frombuffer(b"\x01 The birch canoe slid on the smooth planks.", dtype=np.uint8).astype(np.int32)
    lib = ttship.lib()
    outs = []
    no_epi = ttship.FUSE_ALL & ~8  # TTS_FUSE_EPI off: the MLP's SILU and MUL run as their own launches
    for pro, slab, fuse in ((0, 0, 0), (0, 1, no_epi), (1, 1, ttship.FUSE_ALL), (1, 0, ttship.FUSE_ALL), (0, 1, ttship.FUSE_ALL)):
        assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_PRO"], pro) == 0
        assert lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_SLAB"], slab) == 0
        hip.set_option(0, fuse)
        g = ttship.Dia(hip.iface(), ttship.dia_config(**WIDE))
        try:
            audio = np.full(9, 1026, dtype=np.int32)
            seq = []
            for s in range(4):
                lg = g.prefill(text, audio) if s == 0 else g.decode(audio)
                seq.append(lg.copy())
                audio = lg.argmax(axis=1).astype(np.int32)
            outs.append(seq)
        finally:
            g.close()
            lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_PRO"], 1)
            lib.tts_hip_set_option(hip.ptr, ttship.OPT["GEMV_Q80_SLAB"], 1)
            hip.set_option(0, ttship.FUSE_ALL)
    for c in range(1, len(outs)):
        for s, (a, b) in enumerate(zip(outs[0], outs[c])):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (c, s, np.abs(a - b).max())
