#!/usr/bin/env python3
"""Throughput bench: Parler-TTS-mini v1, Q4_K decoder, autoregressive decode on MI355X.

One "step" = one AR decode step (build_parler_graph + compute + greedy sample) for every prompt of
this rank's shard of the prompt batch (default 8 prompts per GPU = the 64-prompt batch over 8 GPUs,
weak scaling).  Each step produces 512 samples @ 44.1 kHz = 11.61 ms of audio and 9 codec tokens
per prompt.  value = audio-seconds produced by all ranks / wall seconds (RTF^-1).

Multi-GPU: one process per GPU (torchrun); prompts shard with no data-path collective; RCCL
(backend "nccl") carries only the barrier / max-over-ranks timing reduction and the final token
gather (the codec-token stream every rank produced, gathered to rank 0).
"""
import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402

SAMPLES_PER_STEP = 512          # DAC hop: one Parler step = 512 samples
SAMPLE_RATE = 44100.0
HEADS = 9
HBM_PEAK_GBS = 8000.0           # MI355X spec (MI355X_MICROARCH.md chip table)

HARVARD = [  # examples/perf_battery/perf_battery.cpp:25-56 (first sentences), token ids derived from bytes
    "The birch canoe slid on the smooth planks.",
    "Glue the sheet to the dark blue background.",
    "It's easy to tell the depth of a well.",
    "These days a chicken leg is a rare dish.",
    "Rice is often served in round bowls.",
    "The juice of lemons makes fine punch.",
    "The box was thrown beside the parked truck.",
    "The hogs were fed chopped corn and garbage.",
]


def prompt_tokens(batch, n, vocab, offset=0):
    """Synthetic prompt ids; row b is global prompt (offset + b), so a rank's shard equals the
    matching rows of the whole batch."""
    out = np.zeros((batch, n), dtype=np.int32)
    for b in range(batch):
        g = b + offset
        s = HARVARD[g % len(HARVARD)].encode()
        for i in range(n):
            out[b, i] = (s[i % len(s)] * 131 + i * 7 + g) % vocab
    return out


def dist_init(backend="nccl"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        return rank, world, local, dist
    return rank, world, local, None


def _comm_device(dist, local):
    return f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu"


def barrier_sync(dist, be):
    if be is not None:
        be.sync()
    if dist is not None:
        import torch
        dist.barrier()
        if dist.get_backend() == "nccl":
            torch.cuda.synchronize()


def max_over_ranks(dist, local, dt):
    """Wall time of the slowest rank (the job finishes when the last shard does)."""
    if dist is None:
        return dt
    import torch
    t = torch.tensor([dt], device=_comm_device(dist, local), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_tokens(dist, rank, world, local, toks):
    """The one cross-rank data exchange: every rank's codec tokens [batch, steps, heads] to rank 0,
    concatenated along the prompt axis in global prompt order.  Returns None on ranks != 0."""
    if dist is None:
        return toks
    import torch
    g = torch.from_numpy(np.ascontiguousarray(toks).astype(np.int64)).to(_comm_device(dist, local))
    parts = [torch.empty_like(g) for _ in range(world)] if rank == 0 else None
    dist.gather(g, parts, dst=0)
    if rank != 0:
        return None
    return np.concatenate([p.cpu().numpy() for p in parts], axis=0).astype(np.int32)


def cpu_baseline(args, n_threads):
    """Oracle (C restatement of ggml-cpu) running the same Parler step graph on host cores."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import py_oracle
    cfg = ttship.parler_config(batch=1, max_ctx=args.ctx + 64)
    p = ttship.Parler(py_oracle.iface(n_threads), cfg)
    try:
        p.prefill(prompt_tokens(1, 8, cfg.prompt_vocab))
        p.generate(1)
        steps, t0 = 0, time.perf_counter()
        while steps < args.cpu_steps and (steps < 2 or time.perf_counter() - t0 < args.cpu_seconds):
            p.generate(1)
            steps += 1
        dt = time.perf_counter() - t0
    finally:
        p.close()
    audio = steps * SAMPLES_PER_STEP / SAMPLE_RATE
    return {"value": audio / dt, "unit": "audio-sec/wall-sec", "cores": n_threads, "kind": "port",
            "sample": f"{steps} Parler-mini Q4_K decode steps, batch 1, KV length ~10 "
                      f"(oracle/ggml_ref.c, C restatement of ggml-cpu scalar paths; reference ggml-cpu unbuildable offline)",
            "codec_tokens_per_s": steps * HEADS / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="prompts per GPU (64-prompt batch / 8 GPUs)")
    ap.add_argument("--ctx", type=int, default=448, help="KV length when timing starts (prompt prefill)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-steps", type=int, default=400)
    ap.add_argument("--no-fusion", action="store_true")
    ap.add_argument("--graphs", type=int, default=1, help="replay each step as a HIP graph (1) or launch eagerly (0)")
    args = ap.parse_args()

    rank, world, local, dist = dist_init()
    be = ttship.HipBackend(local)
    if args.no_fusion:
        be.set_option(0, 0)
    be.set_option(2, args.graphs)
    cfg = ttship.parler_config(batch=args.batch, max_ctx=max(4096, args.ctx + args.steps + args.warmup + 8),
                               arena_bytes=4 << 30)
    runner = ttship.Parler(be.iface(), cfg)
    # text-prompt pass to reach the measured KV length
    runner.prefill(prompt_tokens(args.batch, args.ctx, cfg.prompt_vocab, offset=rank * args.batch))
    runner.generate(args.warmup)
    barrier_sync(dist, be)

    runner.host_stats(reset=True)
    t0 = time.perf_counter()
    toks = runner.generate(args.steps)
    barrier_sync(dist, be)
    dt = time.perf_counter() - t0
    host = runner.host_stats(reset=True)
    dt = max_over_ranks(dist, local, dt)
    gather_tokens(dist, rank, world, local, toks)

    total_prompts = args.batch * world
    audio_s = total_prompts * args.steps * SAMPLES_PER_STEP / SAMPLE_RATE
    value = audio_s / dt
    tokens_per_s = total_prompts * args.steps * HEADS / dt

    # ---- roofline of the dominant kernel (Q4_K dequant-GEMV), HIP events on the backend stream ----
    be.set_option(1, 1)
    be.gemv_stats(-1, reset=True)
    runner.generate(max(5, args.steps // 5))
    ms, launches, nbytes = be.gemv_stats(ttship.Q4_K, reset=True)
    be.set_option(1, 0)
    gemv_avg_us = 1000.0 * ms / max(launches, 1)
    gemv_gbs = (nbytes / max(launches, 1)) / (gemv_avg_us * 1e-6) / 1e9 if launches else 0.0

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            ncpu = min(16, len(os.sched_getaffinity(0)))
            cpu = cpu_baseline(args, ncpu)
        result = {
            "metric": "audio-sec/wall-sec (RTF^-1), Parler-TTS-mini v1 Q4_K AR decode",
            "value": round(value, 3),
            "unit": "audio-sec/wall-sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "q4_K weights x q8_K activations (int dot), f32 accumulate",
            "data": "synthetic (deterministic Q4_K/F32 weights of Parler-mini v1 shapes; token ids from Harvard sentences)",
            "config": {"workload": "Parler-TTS-mini-v1 Q4_K decoder, greedy AR decode (BASELINE configs[2])",
                       "model": "parler-tts-mini-v1", "prompts_per_gpu": args.batch, "global_batch": total_prompts,
                       "kv_len_start": args.ctx, "parallelism": f"dp{world} (prompt shards)",
                       "graph_nodes_per_step": runner.last_graph_nodes()},
            "codec_tokens_per_s": round(tokens_per_s, 1),
            "host_us_per_step": host,
            "roofline": {"bound": "hbm", "achieved": round(gemv_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gemv_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "k_gemv_q4_K", "avg_launch_us": round(gemv_avg_us, 3),
                         "bytes_per_launch": round(nbytes / max(launches, 1), 1), "launches_sampled": launches},
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    runner.close()
    be.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
