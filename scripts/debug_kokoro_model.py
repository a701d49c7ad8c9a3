"""Kokoro end to end, HIP vs oracle, named-node diff of the main graph (debugging aid).
Usage: python scripts/debug_kokoro_model.py [tiny|82m] [n_tokens]"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in ("tts.cpp_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))
import py_oracle  # noqa: E402
import ttship  # noqa: E402
from test_kokoro_model_cpu import TINY, tokens  # noqa: E402

NAMES = ["shared_lstm", "f0_out", "n_out", "text_encoder", "asr", "encoder_block", "decoder_block.0", "decoder_block.1",
         "decoder_block.2", "decoder_block.3", "decoder_out", "uv_noise", "sine_source", "har_spec", "up.0", "noise_conv.0",
         "noise_res.0", "level.0", "up.1", "level.1", "conv_post", "after_res_gen"]


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "tiny"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    reuse = len(sys.argv) > 3 and sys.argv[3] == "reuse"
    kw = dict(TINY) if which == "tiny" else dict(max_tokens=16, max_total=64)
    cfg = ttship.kokoro_config(**kw, debug_no_reuse=0 if reuse else 1, arena_bytes=0 if reuse else 2 << 30)
    be = ttship.HipBackend(0)
    g = ttship.Kokoro(be.iface(), cfg)
    o = ttship.Kokoro(py_oracle.iface(16), cfg)
    toks = tokens(n, 0)
    ho, lo = o.durations(toks)
    total = int(lo.sum())
    rand = np.random.default_rng(7).random((cfg.gen.harmonic_num + 1, 600 * total), dtype=np.float32)
    po = o.decode(toks, ho, lo, rand)
    masks = [None, 0] + ([ttship.FUSE_ALL & ~b for b in ttship.FUSE.values()] if reuse else [])
    for fusion in masks:
        if fusion is not None:
            be.set_option(ttship.OPT["FUSION"], fusion)
        pg = g.decode(toks, ho, lo, rand)
        print(f"fusion {'default' if fusion is None else fusion}: pcm max err {float(np.max(np.abs(pg - po))):.3e}")
        if reuse:
            continue
        for nm in NAMES:
            a, b = g.node(nm), o.node(nm)
            if a is None or b is None:
                print(f"  {nm:18s} missing ({a is None}, {b is None})")
                continue
            print(f"  {nm:18s} n={b.size:8d} max err {float(np.max(np.abs(a - b))):.3e} scale {float(np.max(np.abs(b))):.3e}")
    g.close()
    o.close()
    be.close()


if __name__ == "__main__":
    main()
