"""The bench's batched prompt pass alone (R runners of B ragged prompts each, the perf_battery sentences):
per-pass wall time and the runner's host split, over several passes.  Run under rocprofv3 --kernel-trace
for the kernels of one pass.  With NAME=OPT:VAL[,OPT:VAL] variants, the passes alternate between them
(interleaved A/B in one process).  Usage: prompt_pass_probe.py [B] [passes] [replicas] [variants ...]"""
import pathlib
import statistics
import sys
import threading
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "tts.cpp_amd"))
import ttship  # noqa: E402
from bench import HARVARD, sentence_tokens  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    variants = []
    for v in sys.argv[4:]:
        name, _, spec = v.partition("=")
        variants.append((name, [(ttship.OPT[k], int(val)) for k, _, val in (kv.partition(":") for kv in filter(None, spec.split(",")))]))
    if not variants:
        variants = [("default", [])]
    cfg = ttship.parler_config(batch=B, max_ctx=256)
    toks = [sentence_tokens(HARVARD[g % len(HARVARD)], cfg.prompt_vocab) for g in range(B * R)]
    bes = [ttship.HipBackend(0) for _ in range(R)]
    runs = [ttship.Parler(b.iface(), cfg) for b in bes]

    def one(r):
        runs[r].reset()
        runs[r].prefill_ragged(toks[r * B:(r + 1) * B])
        bes[r].sync()

    def timed():
        t0 = time.perf_counter()
        th = [threading.Thread(target=one, args=(r,)) for r in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return 1000 * (time.perf_counter() - t0)

    ms = {name: [] for name, _ in variants}
    for name, opts in variants:  # warm every variant's kernels
        for b in bes:
            for k, val in opts:
                b.set_option(k, val)
        timed()
    runs[0].host_stats(reset=True)
    for _ in range(passes):
        for name, opts in variants:
            for b in bes:
                for k, val in opts:
                    b.set_option(k, val)
            ms[name].append(timed())
    print(f"B {B} x {R} replicas, lengths {min(map(len, toks))}-{max(map(len, toks))}")
    for name, v in ms.items():
        print(f"  {name:10s} ms per pass median {statistics.median(v):7.3f} min {min(v):7.3f}  {[round(x, 2) for x in sorted(v)]}")
    print("host us per pass (runner 0):", runs[0].host_stats(reset=True))
    for r in runs:
        r.close()
    for b in bes:
        b.close()


if __name__ == "__main__":
    main()
