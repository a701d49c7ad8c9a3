"""HIP planner's view of the Kokoro-82M graphs built on the CPU oracle (no device): fusion counts,
and with TTS_PLAN_DEBUG=1 the reasons chains stay unfused.  Usage: plan_kokoro.py [n_tokens]"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in ("tts.cpp_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))
import py_oracle  # noqa: E402
import ttship  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cfg = ttship.kokoro_config(max_tokens=max(16, n), max_total=12 * max(16, n))
    k = ttship.Kokoro(py_oracle.iface(8), cfg)
    t = np.zeros(n, np.int32)
    t[1:-1] = 5 + np.arange(n - 2)
    h, lens = k.durations(t)
    print("durations graph:", k.plan_stats(0), k.last_graph_nodes(0), flush=True)
    k.decode(t, h, lens)
    print("main graph:", k.plan_stats(1), k.last_graph_nodes(1), "frames", int(lens.sum()), flush=True)
    k.close()


if __name__ == "__main__":
    main()
