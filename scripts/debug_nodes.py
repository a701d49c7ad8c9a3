"""Debug: run the same Parler step on GPU (fusion off) and oracle, report the first differing node."""
import sys
import numpy as np
sys.path.insert(0, "tts.cpp_amd"); sys.path.insert(0, "oracle")
import ttship, py_oracle
B = int(sys.argv[1]) if len(sys.argv) > 1 else 3
TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=96,
            prompt_vocab=512, max_positions=128, batch=B, debug_no_reuse=1)
hip = ttship.HipBackend(0)
hip.set_option(0, 0)
g = ttship.Parler(hip.iface(), ttship.parler_config(**TINY))
c = ttship.Parler(py_oracle.iface(8), ttship.parler_config(**TINY))
prompt = (np.arange(6 * B, dtype=np.int32).reshape(B, 6) * 41) % 512
for phase in ("prefill", "decode"):
    if phase == "prefill":
        g.prefill(prompt); c.prefill(prompt)
    else:
        t = np.full((B, 9), 7, dtype=np.int32); g.decode(t); c.decode(t)
    n = g.last_graph_nodes()
    bad = 0
    for i in range(n):
        og, _, neg, dg = g.node(i)
        oc, _, nec, dc = c.node(i)
        if dg is None or dc is None:
            continue
        if not np.array_equal(dg.view(np.uint32), dc.view(np.uint32)):
            d = np.abs(dg.astype(np.float64) - dc)
            print(f"{phase}: node {i} {og} ne={neg} differs: n_diff={np.sum(d > 0)} max={d.max():.3e}")
            bad += 1
            if bad >= 6:
                break
    print(phase, "nodes", n, "first diffs listed:", bad)
