"""Host cost of one short DAC-44k decode: wall ms per decode with HIP-graph recording on / off, and
the device-only time (the same decode's kernels, timed by events around the compute call)."""
import json, pathlib, sys, time
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402
import torch  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 20
SPLITS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else []  # CONV_SPLIT targets to compare
be = ttship.HipBackend(0)
cfg = ttship.dac_config(max_frames=T)
dac = ttship.Dac(be.iface(), cfg)
codes = np.random.default_rng(0).integers(0, cfg.codebook_size, size=(T, cfg.n_codebooks))
for graphs in (1, 0, 1):
    be.set_option(ttship.OPT["GRAPHS"], graphs)
    for _ in range(3):
        dac.decode(codes)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter(); dac.decode(codes); ts.append(time.perf_counter() - t0)
    print(json.dumps({"frames": T, "graphs": graphs, "ms_min": round(1e3 * min(ts), 3), "ms_med": round(1e3 * float(np.median(ts)), 3)}), flush=True)
ref = dac.decode(codes).copy()
for sp in SPLITS:
    be.set_option(ttship.OPT["CONV_SPLIT"], sp)
    for _ in range(3):
        pcm = dac.decode(codes)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter(); pcm = dac.decode(codes); ts.append(time.perf_counter() - t0)
    print(json.dumps({"frames": T, "conv_split": sp, "ms_min": round(1e3 * min(ts), 3), "ms_med": round(1e3 * float(np.median(ts)), 3),
                      "max_abs_vs_default": float(np.max(np.abs(pcm - ref)))}), flush=True)
dac.close()
