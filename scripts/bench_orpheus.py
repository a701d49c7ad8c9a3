"""Orpheus-3B Q4_K decode throughput on one GPU (BASELINE configs[4] per-GPU shard: 8 prompts).

Synthetic weights in the exact Orpheus shapes (all matrices Q4_K, incl. embedding and the 156 940-row
head), prompt prefill, then timed greedy AR steps with device sampling.  Prints one JSON line:
tokens/s, audio-s/s (82.03 Orpheus tokens per audio-second) and the dequant-GEMV
roofline from in-packet HIP events over profiled steps.
usage: bench_orpheus.py [batch] [steps] [prompt_len] [layers]"""
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402

TOK_PER_AUDIO_S = 82.03


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    n_prompt = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    kw = {"n_layers": int(sys.argv[4])} if len(sys.argv) > 4 else {}
    be = ttship.HipBackend(0)
    if os.environ.get("TTS_BENCH_GRAPHS") is not None:  # 0: eager launches (rocprofv3 kernel traces)
        be.set_option(ttship.OPT["GRAPHS"], int(os.environ["TTS_BENCH_GRAPHS"]))
    for env, opt in (("TTS_BENCH_KS", "GEMV_KS"), ("TTS_BENCH_TILE_BYTES", "Q4K_TILE_BYTES")):
        if os.environ.get(env) is not None:
            be.set_option(ttship.OPT[opt], int(os.environ[env]))
    t0 = time.perf_counter()
    cfg = ttship.orpheus_config(batch=B, max_ctx=n_prompt + steps + 64, arena_bytes=1 << 30, **kw)
    o = ttship.Orpheus(be.iface(), cfg)
    t_load = time.perf_counter() - t0
    prompt = (np.arange(B * n_prompt, dtype=np.int32).reshape(B, n_prompt) * 7919 + 128000) % cfg.vocab_size
    lg = o.prefill(prompt)
    first = lg.argmax(axis=1).astype(np.int32)
    toks = o.generate(first, 4)  # warm (plans, code objects)
    be.sync()
    t0 = time.perf_counter()
    toks = o.generate(toks[:, -1], steps)
    be.sync()
    dt = time.perf_counter() - t0
    # profiled steps: in-packet events around every quantized GEMV launch
    be.set_option(ttship.OPT["PROFILE_GEMV"], 1)
    be.gemv_stats(-1, reset=True)
    o.generate(toks[:, -1], 8)
    ms, launches, nbytes = be.gemv_stats(ttship.Q4_K, reset=True)
    be.set_option(ttship.OPT["PROFILE_GEMV"], 0)
    avg_us = 1000.0 * ms / max(launches, 1)
    gbs = nbytes / max(launches, 1) / (avg_us * 1e-6) / 1e9
    print(json.dumps({
        "workload": f"Orpheus-3B Q4_K greedy decode, {B} prompts, {cfg.n_layers} layers, prompt {n_prompt}",
        "tokens_per_s": round(B * steps / dt, 1), "audio_sec_per_s": round(B * steps / dt / TOK_PER_AUDIO_S, 3),
        "ms_per_step": round(1000 * dt / steps, 3), "graph_nodes": o.last_graph_nodes(),
        "weight_GB": round(o.weight_bytes() / 1e9, 3), "load_s": round(t_load, 1),
        "gemv_roofline": {"kernel": "k_gemv_q4K_mf / k_gemv_q4_K", "avg_launch_us": round(avg_us, 2),
                          "bytes_per_launch": round(nbytes / max(launches, 1)), "achieved_GBps": round(gbs, 1),
                          "frac": round(gbs / 8000.0, 4), "launches": launches},
        "step_GBps_weights": round(o.weight_bytes() / (dt / steps) / 1e9, 1)}), flush=True)
    o.close()
    be.close()


if __name__ == "__main__":
    main()
