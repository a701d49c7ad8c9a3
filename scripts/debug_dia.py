"""Dia GPU-vs-oracle attention check over head sizes (debug)."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
import py_oracle  # noqa: E402
import ttship  # noqa: E402
from test_dia_gpu import TINY  # noqa: E402

hip = ttship.HipBackend(0)
text = np.frombuffer(b"\x01 The birch canoe slid on the smooth planks. \x02 Glue the sheet.", dtype=np.uint8).astype(np.int32)[:32]
audio = np.full(9, 1026, dtype=np.int32)
cfgs = {"hd32": TINY, "hd64": dict(TINY, encoder_attn_heads=2, decoder_attn_heads=2, head_size=64),
        "hd128": dict(TINY, encoder_attn_heads=1, decoder_attn_heads=1, decoder_query_heads=1, head_size=128),
        "wide1": dict(n_encoder_layers=1, n_decoder_layers=1, max_generation_size=16)}
for name, kw in cfgs.items():
    c = ttship.Dia(py_oracle.iface(16), ttship.dia_config(**kw))
    g = ttship.Dia(hip.iface(), ttship.dia_config(**kw))
    t = text[: c.cfg.max_encoder_context_length]
    lc0, lg0 = c.prefill(t, audio), g.prefill(t, audio)
    a = lc0.argmax(axis=1).astype(np.int32)
    lc1, lg1 = c.decode(a), g.decode(a)
    print(name, "prefill", float(np.abs(lg0 - lc0).max()), "decode", float(np.abs(lg1 - lc1).max()), "max", float(np.abs(lc0).max()), flush=True)
    g.close()
    c.close()
