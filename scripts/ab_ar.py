"""Interleaved A/B of backend options on the 64-prompt AR step (2 replicas x 32 lock-step prompts), in ONE
process: the replicas are prefilled and warmed once, then blocks of timed steps alternate between the
variants (each block after a few untimed steps that re-record the step graphs), so clock state, box and
KV length drift hit every variant alike.  Prints one JSON line per variant: median / min ms per step.

usage: python3 scripts/ab_ar.py [--ctx 448] [--blocks 6] [--steps 12] NAME=OPT:VAL[,OPT:VAL] ...
       (every variant sets every option any variant touches; OPT is a ttship.OPT key, e.g. ATTN_PV_MP:2)"""
import argparse
import json
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import bench  # noqa: E402
import ttship  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=448)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    variants = []
    for v in a.variants:
        name, _, spec = v.partition("=")
        opts = []
        for kv in filter(None, spec.split(",")):
            k, _, val = kv.partition(":")
            opts.append((ttship.OPT[k], int(val)))
        variants.append((name, opts))
    keys = sorted({k for _, o in variants for k, _ in o})
    for name, o in variants:  # every variant sets every option any variant touches (no read-back API)
        if sorted(k for k, _ in o) != keys:
            raise SystemExit(f"variant {name} must set every option the variants touch")
    total_steps = 4 + a.blocks * len(variants) * (a.steps + 2)
    args = argparse.Namespace(steps=total_steps, warmup=0, ctx=a.ctx, cu_partition=0, dac_conv_split=None, dac_batch=None)
    R = a.replicas
    reps, _, _ = bench.parler_replicas(args, a.prompts, R, 0, lambda: ttship.HipBackend(0), None)

    def gen(n):
        bench.run_replicas(lambda r: (reps[r][1].generate(n), reps[r][0].sync()), R)

    gen(4)
    res = {name: [] for name, _ in variants}
    for b in range(a.blocks):
        for name, opts in variants:
            for rb, _, _ in reps:
                for k, val in opts:
                    rb.set_option(k, val)
            gen(2)  # re-record with this variant's kernels
            t0 = time.perf_counter()
            gen(a.steps)
            res[name].append(1000.0 * (time.perf_counter() - t0) / a.steps)
    for name, _ in variants:
        v = res[name]
        print(json.dumps({"variant": name, "ms_median": round(statistics.median(v), 4), "ms_min": round(min(v), 4),
                          "blocks": [round(x, 3) for x in v], "ctx": a.ctx, "prompts": a.prompts, "replicas": R}), flush=True)
    for rb, rr, _ in reps:
        rr.close()
        rb.close()


if __name__ == "__main__":
    main()
