"""Debug: decode attention through graph_compute with VMM-backed buffers, per mode and P; prints how far
the GPU output is from the oracle's (tests/test_attn_gpu.py's graph)."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in ("tts.cpp_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))
import numpy as np
import ttship
import test_attn_gpu as T

hip = ttship.HipBackend(0)
order = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fused:1024", "fused:700", "split:1024", "rows:1024", "fused:1024"]
for spec in order:
    mode, P = spec.split(":")
    P = int(P)
    hd, H, Hk, B = 64, 4, 4, 1
    T.set_mode(hip, mode)
    rng = np.random.default_rng(P * 7 + hd)
    max_ctx = P + 40
    q = rng.standard_normal((B, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, Hk * hd)).astype(np.float32)
    vc = rng.standard_normal((B, Hk * hd, max_ctx)).astype(np.float32)
    mask = np.zeros(P, np.float32)
    mask[P // 3] = -np.inf
    g1, g2 = T.nd.Graph(), T.nd.Graph()
    o1 = T.build(g1, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    o2 = T.build(g2, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    g1.run_hip(hip)
    g2.run_oracle(n_threads=8)
    T.set_mode(hip, "default")
    a, b = g1.node_array(o1), g2.node_array(o2)
    print(f"{mode} P={P}: max|d| {np.abs(a - b).max():.3e} zeros {np.mean(a == 0):.3f}", flush=True)
