"""Debug: a coalesced step (2 one-prompt runners from 2 threads), runners freed, then decode attention on
fresh VMM buffers (tests/test_attn_gpu.py's graph) -- does a reused window range read stale memory?"""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in ("tts.cpp_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))
import numpy as np
import ttship
import test_coalesce_gpu as C
import test_attn_gpu as T

cfg = ttship.parler_config(batch=1, **C.TINY)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
bes = [ttship.HipBackend(0) for _ in range(n)]
got = C.serve([b.iface(reference_flow=True) for b in bes], cfg, [C.prompt(r) for r in range(n)], 6)
for b in bes:
    b.close()
print("coalesce", ttship.coalesce_stats(0), flush=True)
hip = ttship.HipBackend(0)
for P in (700, 1024, 1500, 1024):
    hd, H, Hk, B = 64, 4, 4, 1
    T.set_mode(hip, "fused")
    rng = np.random.default_rng(P * 7 + hd)
    max_ctx = P + 40
    q = rng.standard_normal((B, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, Hk * hd)).astype(np.float32)
    vc = rng.standard_normal((B, Hk * hd, max_ctx)).astype(np.float32)
    mask = np.zeros(P, np.float32)
    g1, g2 = T.nd.Graph(), T.nd.Graph()
    o1 = T.build(g1, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    o2 = T.build(g2, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    g1.run_hip(hip)
    g2.run_oracle(n_threads=8)
    a, b = g1.node_array(o1), g2.node_array(o2)
    print(f"fused P={P}: max|d| {np.abs(a - b).max():.3e} zeros {np.mean(a == 0):.3f}", flush=True)
