"""Debug: Kokoro generator node-by-node HIP vs oracle (debug_no_reuse, fusion off), printing the
first nodes that differ.  Usage: python scripts/kokoro_diff.py [fusion_mask]"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in ("tts.cpp_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))
import py_oracle  # noqa: E402
import ttship  # noqa: E402
from test_kokoro_cpu import inputs  # noqa: E402


def main():
    fusion = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    be = ttship.HipBackend(0)
    be.set_option(0, fusion)
    cfg = ttship.kokoro_gen_config(in_channels=32, style_dim=16, max_frames=16, debug_no_reuse=1, arena_bytes=256 << 20)
    args = inputs(cfg, 4, 0)
    kg = ttship.KokoroGenerator(be.iface(), cfg)
    ko = ttship.KokoroGenerator(py_oracle.iface(8), cfg)
    a, b = kg.run(*args), ko.run(*args)
    print("pcm maxdiff", float(np.max(np.abs(a - b))))
    shown = 0
    for i in range(kg.last_graph_nodes()):
        op, ty, ne, g = kg.node_at(i)
        _, _, _, o = ko.node_at(i)
        if g is None or o is None or ty != 0:
            continue
        d = float(np.max(np.abs(g - o))) if g.size else 0.0
        if d > 0:
            print(i, op, ne, "maxdiff", d, "scale", float(np.max(np.abs(o))), "nmis", int(np.sum(g != o)))
            shown += 1
            if shown > 25:
                break
    be.close()


if __name__ == "__main__":
    main()
