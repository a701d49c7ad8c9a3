"""GEMV micro-benchmark (raw tts_hip_gemv entry, HIP-event timed on the backend stream).

Shapes: the Parler-mini decode matrices, Orpheus-3B / Dia sizes, at M = 1 and 8 columns.
Prints one JSON line per shape with avg us per launch and algorithmic GB/s.
"""
import json
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402

SHAPES = [  # (name, type, K, N)
    ("parler_qkvo", ttship.Q4_K, 1024, 1024),
    ("parler_fc1", ttship.Q4_K, 1024, 4096),
    ("parler_fc2", ttship.Q4_K, 4096, 1024),
    ("orpheus_q", ttship.Q4_K, 3072, 3072),
    ("orpheus_up", ttship.Q4_K, 3072, 8192),
    ("orpheus_down", ttship.Q4_K, 8192, 3072),
    ("orpheus_head", ttship.Q4_K, 3072, 156940),
    ("dia_ffn", ttship.Q8_0, 2048, 8192),
    ("parler_head_f32", ttship.F32, 1024, 1088 * 9),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    mlist = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 8]
    tiled = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # 1: Q4_K in the tile layout (matrix-core kernel)
    only = sys.argv[4].split(",") if len(sys.argv) > 4 else None
    mr_tiles = None
    hip = ttship.HipBackend(0)
    dbg = int(sys.argv[6]) if len(sys.argv) > 6 else 0  # TTS_HIP_OPT_GEMV_DEBUG phase study
    hip.set_option(ttship.OPT["GEMV_DEBUG"], dbg)
    # cold: cycle through enough weight copies (>= 512 MiB) that every launch streams from HBM, as in a
    # decode step (the Infinity Cache holds 256 MiB); kernel selection from the environment
    cold = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    for opt in ("GEMV_UNIQUE", "GEMV_KS"):
        if os.environ.get(opt) is not None:
            hip.set_option(ttship.OPT[opt], int(os.environ[opt]))
    L = ttship.lib()
    rng = np.random.default_rng(0)
    for name, wt, K, N in SHAPES:
        if only and name not in only:
            continue
        wbytes = ttship.row_size(wt, K) * N
        w = rng.integers(0, 256, size=wbytes, dtype=np.uint8)
        if wt == ttship.Q4_K:  # keep d/dmin finite: small fp16 in the block headers
            blk = w.reshape(-1, 144)
            blk[:, 0:2] = np.frombuffer(np.float16(1e-3).tobytes(), dtype=np.uint8)
            blk[:, 2:4] = np.frombuffer(np.float16(1e-3).tobytes(), dtype=np.uint8)
        elif wt == ttship.Q8_0:
            blk = w.reshape(-1, 34)
            blk[:, 0:2] = np.frombuffer(np.float16(1e-3).tobytes(), dtype=np.uint8)
        else:
            w = (rng.standard_normal(K * N).astype(np.float32) * 0.02).view(np.uint8)
        flags = 0
        if tiled and wt == ttship.Q4_K:  # random bytes are valid in any layout; only the flag matters
            flags = 32
            if N % 4:
                continue
        ncopy = max(1, min(64, -(-(512 << 20) // w.nbytes))) if cold else 1
        dws = [hip.alloc(w.nbytes) for _ in range(ncopy)]
        for d in dws:
            hip.set(d, w)
        for M in mlist:
            x = rng.standard_normal((M, K)).astype(np.float32)
            dx = hip.alloc(x.nbytes)
            dy = hip.alloc(4 * M * N)
            hip.set(dx, x)
            for c in range(3):
                L.tts_hip_gemv_ex(hip.ptr, wt, dws[c % ncopy], dx, dy, K, N, M, flags)
            hip.sync()
            hip.set_option(1, 1)
            hip.gemv_stats(-1, reset=True)
            for c in range(reps):
                L.tts_hip_gemv_ex(hip.ptr, wt, dws[c % ncopy], dx, dy, K, N, M, flags)
            ms, n, nbytes = hip.gemv_stats(wt, reset=True)
            hip.set_option(1, 0)
            us = 1000.0 * ms / n
            print(json.dumps({"shape": name, "type": ttship.lib().tts_type_name(wt).decode(), "K": K, "N": N, "M": M,
                              "weight_MB": round(wbytes / 1e6, 3), "tiled": bool(tiled and wt == ttship.Q4_K), "dbg": dbg, "cold": cold,
                              "avg_us": round(us, 2),
                              "GBps": round(nbytes / n / (us * 1e-6) / 1e9, 1)}), flush=True)
            hip.free(dx)
            hip.free(dy)
        for d in dws:
            hip.free(d)
    hip.close()


if __name__ == "__main__":
    main()
