"""Decode-attention micro-benchmark at Parler (hd 64, H 16, B 8) and Orpheus (hd 128, H 24, B 1; the
Orpheus runner hands attention its GQA copies of K / V, so Hk = H here)
shapes: the unfused reference chain (tests/test_attn_gpu.py `build`) through tts_hip_graph_compute,
which the planner fuses into one attention item, repeated `reps` times with the split kernels on and
off.  Wall time per call after a device sync; run under rocprofv3 --kernel-trace for kernel times.
Prints one JSON line per (shape, P, split) with the algorithmic KV bytes and GB/s of the wall time."""
import ctypes
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for d in ("tts.cpp_amd", "tests", "oracle"):
    sys.path.insert(0, str(ROOT / d))
import ttship  # noqa: E402
import nodes as nd  # noqa: E402
from test_attn_gpu import build  # noqa: E402


def run(hip, P, hd, H, Hk, B, reps, split):
    rng = np.random.default_rng(P)
    max_ctx = 4096
    q = rng.standard_normal((B, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, Hk * hd), dtype=np.float32)
    vc = rng.standard_normal((B, Hk * hd, max_ctx), dtype=np.float32)
    mask = np.zeros(P, np.float32)
    g = nd.Graph()
    build(g, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    dev = {}
    for t in g.tensors:
        if id(t) in g.arrays:
            buf = g.arrays[id(t)]
            d = hip.alloc(buf.nbytes)
            hip.set(d, buf)
            dev[id(t)] = d
            t.data = d
    for t in g.tensors:
        if getattr(t, "_root", None) is not None:
            t.data = dev[id(t._root)] + t._root_offs
    hip.set_option(ttship.OPT["ATTN_FUSED"], ttship.ATTN_FUSED_ON if split == "fused" else 0)
    hip.set_option(ttship.OPT["ATTN_SPLIT"], ttship.ATTN_SPLIT_DEFAULT if split == "split" else 0)
    ptrs = g.node_ptrs()
    L = ttship.lib()
    def compute():
        st = L.tts_hip_graph_compute(hip.ptr, ptrs, len(g.nodes))
        if st != 0:
            raise RuntimeError(f"tts_hip_graph_compute failed {st} (P {P}, hd {hd}, H {H}, Hk {Hk}, B {B}, {split})")
    for _ in range(3):
        compute()
    hip.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        compute()
    hip.sync()
    dt = (time.perf_counter() - t0) / reps
    for d in dev.values():
        hip.free(d)
    hip.set_option(ttship.OPT["ATTN_SPLIT"], ttship.ATTN_SPLIT_DEFAULT)
    hip.set_option(ttship.OPT["ATTN_FUSED"], 0)
    kv = 2 * B * Hk * P * hd * 4 if Hk == H else 2 * B * H * P * hd * 4  # bytes the kernel streams
    return {"hd": hd, "H": H, "Hk": Hk, "B": B, "P": P, "split": split, "us_per_call": round(dt * 1e6, 2),
            "kv_MB": round(kv / 1e6, 2), "GBps_wall": round(kv / dt / 1e9, 1)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    hip = ttship.HipBackend(0)
    shapes = [(64, 16, 16, 8), (128, 24, 24, 1)]
    Ps = (448, 900, 1309, 2048)
    if "--many" in sys.argv:  # the many-prompt decode step: Parler at 32 / 64 lock-step prompts
        shapes, Ps = [(64, 16, 16, 32), (64, 16, 16, 64)], (460,)
    modes = ("rows", "split", "fused")
    for a in sys.argv:
        if a.startswith("--P="):  # e.g. --P=460,1200 (with --many: the split pair only)
            Ps, modes = tuple(int(x) for x in a[4:].split(",")), ("split",)
    for (hd, H, Hk, B) in shapes:
        for P in Ps:
            for split in modes:
                print(json.dumps(run(hip, P, hd, H, Hk, B, reps, split)), flush=True)
    hip.close()


if __name__ == "__main__":
    main()
