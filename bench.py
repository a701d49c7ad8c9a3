#!/usr/bin/env python3
"""Throughput bench: Parler-TTS-mini v1 Q4_K on MI355X -- autoregressive decode + DAC decode
(BASELINE.json configs[2], "AR decode + DAC conv_transpose_1d").

A "step" is one AR decode step (build_parler_graph + compute + greedy sample) for every prompt of
this rank's shard of the prompt batch (default 8 prompts per GPU = the 64-prompt batch over 8 GPUs,
weak scaling).  Each step produces 512 samples @ 44.1 kHz = 11.61 ms of audio and 9 codec tokens
per prompt.  After the K timed steps every prompt's K codec frames are decoded to PCM by the DAC-44k
decoder inside the same timed region.  value = audio-seconds produced by all ranks / wall seconds
(RTF^-1) of AR + DAC; the AR-only and DAC-only rates are reported beside it.

Beside the headline line's fields, three more legs of BASELINE.json's configs run on the same GPU:
"kokoro" (configs[1], Kokoro-82M fp16 end to end: durations, decoder, iSTFTNet vocoder), "dia" (configs[3], Dia-1.6B Q8_0 CFG
decode) and "orpheus" (configs[4]'s per-GPU shard, Orpheus-3B Q4_K decode), each with its own rate; the orpheus leg carries the dequant-GEMV
roofline at the sizes where the matrix-core GEMV streams (every Orpheus matrix is >= 4 MiB).

Multi-GPU: one process per GPU (torchrun); prompts shard with no data-path collective; RCCL
(backend "nccl") carries only the barrier / max-over-ranks timing reduction and the final token
gather (the codec-token stream every rank produced, gathered to rank 0).
"""
import argparse
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
# offline rocprofv3 --pmc result (scripts/gpu_pmc.sh): the newest round's
PMC_FILE = max((ROOT / "profiles").glob("r*/pmc_gemv_q4k.json"), default=ROOT / "profiles" / "r01" / "pmc_gemv_q4k.json")
# PMC traffic of the Orpheus leg's matrix-core GEMV (scripts/gpu_pmc_orpheus.sh), newest round first
PMC_FILE_ORPH = max((ROOT / "profiles").glob("r*/pmc_gemv_q4k_kr_orpheus.json"), default=None)

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


def dac_codes(toks, codebook_size):
    """Parler codec tokens [steps, heads] -> DAC input [frames, codebooks].  The synthetic decoder's
    tokens include the delay pattern's BOS / EOS ids (>= 1024); they are folded into the codebook
    range (a trained model's output after the delay is undone is already in range)."""
    return np.ascontiguousarray(toks % codebook_size, dtype=np.int32)


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


def gather_audio(dist, rank, world, local, pcms):
    """The final audio gather: every prompt's PCM to rank 0 in global prompt order.
    An all-gather of the per-prompt sample counts, then a gatherv as point-to-point sends of each
    rank's concatenated samples (RCCL send / recv over xGMI; gloo on CPU).  Returns the list of all
    prompts' PCM on rank 0, None elsewhere."""
    if dist is None:
        return list(pcms)
    import torch
    dev = _comm_device(dist, local)
    lens = torch.tensor([len(p) for p in pcms], dtype=torch.int64, device=dev)
    all_lens = [torch.empty_like(lens) for _ in range(world)]
    dist.all_gather(all_lens, lens)
    flat = torch.from_numpy(np.concatenate(pcms).astype(np.float32)).to(dev)
    if rank != 0:
        dist.send(flat, dst=0)
        return None
    out = []
    for r in range(world):
        n = [int(v) for v in all_lens[r].cpu()]
        if r == 0:
            buf = flat
        else:
            buf = torch.empty(sum(n), dtype=torch.float32, device=dev)
            dist.recv(buf, src=r)
        host = buf.cpu().numpy()
        offs = np.cumsum([0] + n)
        out += [host[offs[i]:offs[i + 1]] for i in range(len(n))]
    return out


def cpu_baseline(args, n_threads):
    """Oracle (C restatement of ggml-cpu) on the GPU leg's workload shape, on host cores: the same
    Parler step graph at the same batch (all of this GPU's prompts in one runner) and the same KV
    length when timing starts (tts_parler_set_position: the prefill is skipped, the step's work is
    the same), then the same DAC graph over a few frames per prompt; rates per audio-second,
    end to end = 1 / (1/AR + 1/DAC)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import py_oracle
    B = args.batch
    cfg = ttship.parler_config(batch=B, max_ctx=args.ctx + 64)
    p = ttship.Parler(py_oracle.iface(n_threads), cfg)
    try:
        p.prefill(prompt_tokens(B, 8, cfg.prompt_vocab))
        p.set_position(args.ctx)
        p.generate(1)
        steps, t0 = 0, time.perf_counter()
        while steps < args.cpu_steps and (steps < 2 or time.perf_counter() - t0 < args.cpu_seconds):
            p.generate(1)
            steps += 1
        dt_ar = time.perf_counter() - t0
        toks = p.generate(2)
    finally:
        p.close()
    frames = 2
    dcfg = ttship.dac_config(max_frames=frames)
    dac = ttship.Dac(py_oracle.iface(n_threads), dcfg)
    try:
        t0 = time.perf_counter()
        for b in range(B):
            dac.decode(dac_codes(toks[b], dcfg.codebook_size))
        dt_dac = time.perf_counter() - t0
    finally:
        dac.close()
    ar = B * steps * SAMPLES_PER_STEP / SAMPLE_RATE / dt_ar
    dac_rate = B * frames * SAMPLES_PER_STEP / SAMPLE_RATE / dt_dac
    return {"value": 1.0 / (1.0 / ar + 1.0 / dac_rate), "unit": "audio-sec/wall-sec", "cores": n_threads, "kind": "port",
            "sample": f"{steps} Parler-mini Q4_K decode steps of {B} prompts at KV length {args.ctx} (the GPU leg's batch and KV "
                      f"length; prefill skipped) + DAC-44k decode of {frames} frames per prompt (oracle/ggml_ref.c, C restatement "
                      f"of ggml-cpu scalar paths; reference ggml-cpu unbuildable offline)",
            "ar_audio_sec_per_s": round(ar, 5), "dac_audio_sec_per_s": round(dac_rate, 5),
            "codec_tokens_per_s": B * steps * HEADS / dt_ar}


def gemv_roofline(be, runner, steps):
    """Dominant kernel (Q4_K dequant-GEMV): algorithmic bytes per launch / its average duration,
    HIP events on the backend stream around each launch during profiled decode steps."""
    be.set_option(1, 1)
    be.gemv_stats(-1, reset=True)
    runner.generate(steps)
    ms, launches, nbytes = be.gemv_stats(ttship.Q4_K, reset=True)
    be.set_option(1, 0)
    avg_us = 1000.0 * ms / max(launches, 1)
    bpl = nbytes / max(launches, 1)
    gbs = bpl / (avg_us * 1e-6) / 1e9 if launches else 0.0
    traffic, src = None, None
    if PMC_FILE.exists():
        pmc = json.loads(PMC_FILE.read_text())
        traffic, src = pmc.get("hbm_bytes_per_launch"), str(PMC_FILE.relative_to(ROOT))
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
            "kernel": "k_gemv_q4_K", "avg_launch_us": round(avg_us, 3), "bytes_per_launch": round(bpl, 1),
            "launches_sampled": launches}


def run_replicas(fn, n):
    """fn(0..n-1) concurrently on host threads (the ctypes calls release the GIL), re-raising errors."""
    if n == 1:
        fn(0)
        return
    import threading
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]


ORPHEUS_TOK_PER_AUDIO_S = 82.03  # 820 Orpheus tokens = 10.0 s of audio


def orpheus_leg(be, args, rank):
    """BASELINE configs[4] per-GPU shard: Orpheus-3B Q4_K (synthetic weights, every matrix incl. the
    156 940-row head in Q4_K), `orpheus_batch` prompts in lockstep, greedy decode with device
    sampling; plus the dequant-GEMV roofline over profiled steps (the tile-layout matrix-core kernel
    carries every matrix >= 4 MiB)."""
    B, steps, n_prompt = args.orpheus_batch, args.orpheus_steps, 32
    cfg = ttship.orpheus_config(batch=B, max_ctx=n_prompt + steps + 64, arena_bytes=1 << 30)
    o = ttship.Orpheus(be.iface(), cfg)
    try:
        prompt = (np.arange(B * n_prompt, dtype=np.int32).reshape(B, n_prompt) * 7919 + 128000 + rank) % cfg.vocab_size
        first = o.prefill(prompt).argmax(axis=1).astype(np.int32)
        toks = o.generate(first, 4)
        be.sync()
        t0 = time.perf_counter()
        toks = o.generate(toks[:, -1], steps)
        be.sync()
        dt = time.perf_counter() - t0
        be.set_option(ttship.OPT["PROFILE_GEMV"], 1)
        be.gemv_stats(-1, reset=True)
        o.generate(toks[:, -1], 8)
        ms, launches, nbytes = be.gemv_stats(ttship.Q4_K, reset=True)
        be.set_option(ttship.OPT["PROFILE_GEMV"], 0)
        avg_us = 1000.0 * ms / max(launches, 1)
        gbs = nbytes / max(launches, 1) / (avg_us * 1e-6) / 1e9 if launches else 0.0
        return {"workload": f"Orpheus-3B Q4_K greedy decode (BASELINE configs[4] per-GPU shard), {B} prompts, "
                            f"prompt {n_prompt} + {steps} timed steps, synthetic weights",
                "tokens_per_s": round(B * steps / dt, 1), "audio_sec_per_s": round(B * steps / dt / ORPHEUS_TOK_PER_AUDIO_S, 3),
                "ms_per_step": round(1000 * dt / steps, 3), "graph_nodes": o.last_graph_nodes(),
                "weight_bytes": o.weight_bytes(),
                "roofline": {"bound": "hbm", "kernel": "k_gemv_q4K_kr (K relay, tile layout, >= 4 MiB; its operand pass k_quant_mf "
                                                      "not included) + k_gemv_q4_K (k / v lane layout)",
                             "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "avg_launch_us": round(avg_us, 3), "bytes_per_launch": round(nbytes / max(launches, 1), 1),
                             "launches_sampled": launches,
                             "traffic_kr": (json.loads(PMC_FILE_ORPH.read_text()).get("hbm_bytes_per_launch") if PMC_FILE_ORPH else None),
                             "traffic_source": str(PMC_FILE_ORPH.relative_to(ROOT)) if PMC_FILE_ORPH else None}}
    finally:
        o.close()


def dia_leg(be, args):
    """BASELINE configs[3]: Dia-1.6B Q8_0 (synthetic weights), encoder step over a Harvard-sentence
    prompt, then timed CFG decoder steps (conditioned + unconditioned in one graph, greedy heads fed
    back).  One step = one 9-codebook DAC frame = 512 samples at 44.1 kHz."""
    d = ttship.Dia(be.iface(), ttship.dia_config(max_generation_size=args.dia_steps + 16))
    try:
        text = np.frombuffer(("\x01 " + HARVARD[0] + " " + HARVARD[1]).encode(), dtype=np.uint8).astype(np.int32)
        t0 = time.perf_counter()
        audio = d.prefill(text, np.full(9, 1026, dtype=np.int32)).argmax(axis=1).astype(np.int32)
        t_enc = time.perf_counter() - t0
        audio = d.generate(audio, 3)[-1]  # warm (plans, code objects)
        be.sync()
        t0 = time.perf_counter()
        d.generate(audio, args.dia_steps)  # device-resident greedy loop
        be.sync()
        dt = time.perf_counter() - t0
        return {"workload": "Dia-1.6B Q8_0 CFG decode (BASELINE configs[3]), 1 prompt, synthetic weights",
                "ms_per_step": round(1000 * dt / args.dia_steps, 3),
                "audio_sec_per_s": round(args.dia_steps * SAMPLES_PER_STEP / SAMPLE_RATE / dt, 3),
                "encoder_step_ms": round(1000 * t_enc, 1), "weight_bytes": d.weight_bytes()}
    finally:
        d.close()


def parler_b1_leg(args, rank, local, new_backend):
    """TTS.cpp's serving shape (examples/server/server.cpp:316-321,885-895): one prompt per runner,
    `b1_replicas` runners, each on its own backend (HIP stream) driven by its own host thread, all
    prefilled to the same KV length; beside the headline's lock-step batches."""
    R, steps = args.b1_replicas, args.b1_steps
    # the same KV capacity rule as the lock-step leg: a multiple of 4 positions keeps every V row
    # 16-B aligned, so P.V takes its vector-load kernel (k_attn_pv<true, ...>)
    cfg = ttship.parler_config(batch=1, max_ctx=max(4096, args.ctx + steps + args.warmup + 64))
    bes = [new_backend() for _ in range(R)]
    runs = [ttship.Parler(b.iface(), cfg) for b in bes]
    try:
        for r, (b, p) in enumerate(zip(bes, runs)):
            p.prefill(prompt_tokens(1, args.ctx, cfg.prompt_vocab, offset=rank * R + r))
            p.generate(args.warmup)
            b.sync()

        def one(r):
            runs[r].generate(steps)
            bes[r].sync()

        t0 = time.perf_counter()
        run_replicas(one, R)
        dt = time.perf_counter() - t0
        return {"workload": f"Parler-mini Q4_K AR decode, {R} runners x 1 prompt (TTS.cpp's server model), KV {args.ctx} -> "
                            f"{args.ctx + steps}", "replicas": R, "batch_per_replica": 1,
                "ms_per_step": round(1000 * dt / steps, 4),
                "ar_audio_sec_per_s": round(R * steps * SAMPLES_PER_STEP / SAMPLE_RATE / dt, 3)}
    finally:
        for p in runs:
            p.close()
        for b in bes:
            b.close()


def kokoro_prompt(g, vocab):
    """Synthetic phoneme ids for global prompt g: a Harvard sentence's bytes mapped into the
    phoneme vocabulary, wrapped in the boundary id 0 as the phonemizer wraps a prompt."""
    s = HARVARD[g % len(HARVARD)].encode()
    ids = [(b * 131 + i * 7 + g) % (vocab - 1) + 1 for i, b in enumerate(s)]
    return np.asarray([0] + ids + [0], dtype=np.int32)


def kokoro_leg(backends, args, rank, dist, local, world):
    """BASELINE configs[1]: Kokoro-82M end to end (kokoro_runner::run: duration graph, host mask
    step, main graph with the iSTFTNet generator) over `kokoro_prompts` Harvard-sentence prompts per
    GPU, synthetic weights.  Each replica backend (its own HIP stream) owns a runner and serves every
    R-th prompt from a host thread, as the server's workers each own a runner
    (examples/server/server.cpp:316-321): one prompt's host-side graph building overlaps another's
    device work."""
    kcfg = ttship.kokoro_config(max_tokens=64, max_total=600, weight_type=ttship.F16)  # configs[1]: Kokoro-82M fp16
    R = len(backends)
    koks = [ttship.Kokoro(b.iface(), kcfg) for b in backends]
    try:
        prompts = [kokoro_prompt(rank * args.kokoro_prompts + i, kcfg.n_vocab) for i in range(args.kokoro_prompts)]
        for k in koks:
            k.run(prompts[0])  # warm (code objects, arena)
        samples = [0] * R

        def serve(r):
            for p in prompts[r::R]:
                samples[r] += koks[r].run(p).shape[0]
            backends[r].sync()

        barrier_sync(dist, backends[0])
        t0 = time.perf_counter()
        run_replicas(serve, R)
        dt = max_over_ranks(dist, local, time.perf_counter() - t0)
        # per-stage split on the first prompt, one runner alone (durations graph vs main graph incl. generator)
        t1 = time.perf_counter()
        hidden, lens = koks[0].durations(prompts[0])
        t2 = time.perf_counter()
        koks[0].decode(prompts[0], hidden, lens)
        t3 = time.perf_counter()
        audio = sum(samples) / kcfg.gen.sample_rate
        return {"workload": f"Kokoro-82M end to end (BASELINE configs[1]): tokens -> durations -> decoder -> iSTFTNet PCM, "
                            f"{args.kokoro_prompts} prompts per GPU served by {R} replica runners, synthetic weights",
                "audio_sec_per_s": round(world * audio / dt, 3), "ms_per_prompt": round(1000.0 * dt / len(prompts), 3),
                "audio_sec_per_gpu": round(audio, 3), "tokens_per_prompt": [int(p.shape[0]) for p in prompts], "replicas": R,
                "first_prompt_ms": {"durations": round(1000 * (t2 - t1), 3), "decode": round(1000 * (t3 - t2), 3),
                                    "frames": int(lens.sum())},
                "graph_nodes": [koks[0].last_graph_nodes(0), koks[0].last_graph_nodes(1)],
                "dtype": "f16 weights (F16 GGUF: matrices and conv kernels, quantize_impl.cpp:14-18), f32 activations, f16-rounded "
                         "mul_mat / conv inputs (ggml vec_dot_type, im2col), f64 accumulate"}
    finally:
        for k in koks:
            k.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=861, help="AR steps per prompt (861 = 10.0 s of audio, SURVEY §8d)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="prompts per GPU (64-prompt batch / 8 GPUs)")
    ap.add_argument("--ctx", type=int, default=448, help="KV length when timing starts (prompt prefill)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-steps", type=int, default=400)
    ap.add_argument("--b1-replicas", type=int, default=8, help="the B=1 leg: this many runners of one prompt each, as "
                    "TTS.cpp's server workers run (0 = skip)")
    ap.add_argument("--b1-steps", type=int, default=100)
    ap.add_argument("--no-fusion", action="store_true")
    ap.add_argument("--no-dac", action="store_true", help="AR decode only")
    ap.add_argument("--attn-split", type=int, default=None, help="TTS_HIP_OPT_ATTN_SPLIT: min KV length for split attention (0 = off)")
    ap.add_argument("--replicas", type=int, default=2, help="concurrent runner replicas per GPU, each on its own "
                    "backend/stream with batch/replicas prompts (the server's worker model)")
    ap.add_argument("--kv-prefetch", type=int, default=None, help="TTS_HIP_OPT_KV_PREFETCH: min KV length (0 = off)")
    ap.add_argument("--kv-prefetch-blocks", type=int, default=None)
    ap.add_argument("--conv-acc", type=int, default=None, help="TTS_HIP_OPT_CONV_F32ACC for the codec / vocoder convs")
    ap.add_argument("--tile-bytes", type=int, default=None, help="TTS_HIP_OPT_Q4K_TILE_BYTES: Q4_K matrices of >= value bytes use the 4-row tile layout (matrix-core GEMVs)")
    ap.add_argument("--attn-pv16", type=int, default=None, help="TTS_HIP_OPT_ATTN_PV16: split P.V requests the whole V slice (P <= 1024) before the softmax (0 = two batches)")
    ap.add_argument("--attn-fused", type=int, default=None, help="TTS_HIP_OPT_ATTN_FUSED: decode attention over >= value keys as one 1024-thread launch (0 = off)")
    ap.add_argument("--gemv-ks", type=int, default=None, help="TTS_HIP_OPT_GEMV_KS: max 16-row tiles of a tile-layout GEMV on the K-split matrix-core kernel (0 = never)")
    ap.add_argument("--gemv-unique", type=int, default=None, help="TTS_HIP_OPT_GEMV_UNIQUE: unique-load Q4_K GEMV (1, default) or octet per (row, column) (0)")
    ap.add_argument("--attn-ks", type=int, default=None, help="TTS_HIP_OPT_ATTN_KS: 128 * value key positions per split-scores workgroup")
    ap.add_argument("--attn-pv8", type=int, default=None, help="TTS_HIP_OPT_ATTN_PV8: 8 output dims per split P.V workgroup (1) or 16 (0)")
    ap.add_argument("--gemv-krelay", type=int, default=None, help="TTS_HIP_OPT_GEMV_KRELAY: K-relay matrix-core GEMV / prefill GEMM (1) or not (0)")
    ap.add_argument("--gemv-q80-pro", type=int, default=None, help="TTS_HIP_OPT_GEMV_Q80_PRO: Q8_0 GEMVs of <= 8 columns quantize / normalize in every workgroup")
    ap.add_argument("--gemv-q80-slab", type=int, default=None, help="TTS_HIP_OPT_GEMV_Q80_SLAB: slab-form Q8_0 GEMV (1) or the row-block kernel (0)")
    ap.add_argument("--gemv-q80-rw", type=int, default=None, help="TTS_HIP_OPT_GEMV_Q80_RW: rows per slab Q8_0 GEMV workgroup (0 = auto)")
    ap.add_argument("--gemm-q8-staged", type=int, default=None, help="TTS_HIP_OPT_GEMM_Q8_STAGED: many-column Q8_0 GEMM kernel (2 = 64x128 staged, 1 = 64x64 staged, 0 = direct)")
    ap.add_argument("--gemv-kr-inkernel", type=int, default=None, help="TTS_HIP_OPT_GEMV_KR_INKERNEL: max K of K-relay GEMVs quantizing in-kernel (0 = operand pass)")
    ap.add_argument("--gemv-nw-min", type=int, default=None, help="TTS_HIP_OPT_GEMV_NW_MIN: minimum waves per lane-layout Q4_K GEMV workgroup")
    ap.add_argument("--graphs", type=int, default=1, help="replay each step as a HIP graph (1) or launch eagerly (0)")
    ap.add_argument("--cu-partition", type=int, default=0, help="TTS_HIP_OPT_CU_PARTITION for the AR replicas: 0 = every "
                    "replica on all CUs, 1 = replica r on the r-th contiguous CU set, 2 = on CUs c with c %% R == r")
    ap.add_argument("--dac-conv-split", type=int, default=None, help="TTS_HIP_OPT_CONV_SPLIT on the DAC workers' backends "
                    "(split convs over extra workgroups; default: the backend's default, on)")
    ap.add_argument("--dac-workers", type=int, default=8, help="concurrent DAC decoders per GPU (each its own backend / "
                    "stream; the AR replicas' backends first): short codec sequences fill few CUs, so several "
                    "prompts decode side by side")
    ap.add_argument("--kokoro-prompts", type=int, default=8, help="Kokoro-82M prompts per GPU, end to end (0 = skip)")
    ap.add_argument("--orpheus-steps", type=int, default=64, help="timed Orpheus-3B decode steps per GPU (0 = skip)")
    ap.add_argument("--orpheus-batch", type=int, default=8, help="Orpheus prompts per GPU (64-prompt batch / 8 GPUs)")
    ap.add_argument("--dia-steps", type=int, default=32, help="timed Dia-1.6B decoder steps per GPU (0 = skip)")
    args = ap.parse_args()

    rank, world, local, dist = dist_init()
    R = args.replicas
    if R < 1 or args.batch % R:
        raise SystemExit(f"--replicas {R} must divide --batch {args.batch}")
    bl = args.batch // R  # prompts per replica
    # the compute arena holds the prompt pass too (attention scores [ctx, ctx, H, prompts]): 4 GiB per 8 prompts
    cfg = ttship.parler_config(batch=bl, max_ctx=max(4096, args.ctx + args.steps + args.warmup + 64),
                               arena_bytes=max(4, (bl + 7) // 8 * 4) << 30)
    def new_backend():
        rb = ttship.HipBackend(local)
        if args.no_fusion:
            rb.set_option(0, 0)
        rb.set_option(2, args.graphs)
        if args.conv_acc is not None:
            rb.set_option(ttship.OPT["CONV_F32ACC"], args.conv_acc)
        if args.attn_split is not None:
            rb.set_option(ttship.OPT["ATTN_SPLIT"], args.attn_split)
        if args.kv_prefetch is not None:
            rb.set_option(ttship.OPT["KV_PREFETCH"], args.kv_prefetch)
        if args.gemv_unique is not None:
            rb.set_option(ttship.OPT["GEMV_UNIQUE"], args.gemv_unique)
        if args.tile_bytes is not None:
            rb.set_option(ttship.OPT["Q4K_TILE_BYTES"], args.tile_bytes)
        if args.gemv_ks is not None:
            rb.set_option(ttship.OPT["GEMV_KS"], args.gemv_ks)
        if args.attn_fused is not None:
            rb.set_option(ttship.OPT["ATTN_FUSED"], args.attn_fused)
        if args.attn_pv16 is not None:
            rb.set_option(ttship.OPT["ATTN_PV16"], args.attn_pv16)
        if args.gemv_krelay is not None:
            rb.set_option(ttship.OPT["GEMV_KRELAY"], args.gemv_krelay)
        if args.gemv_nw_min is not None:
            rb.set_option(ttship.OPT["GEMV_NW_MIN"], args.gemv_nw_min)
        if args.gemv_q80_pro is not None:
            rb.set_option(ttship.OPT["GEMV_Q80_PRO"], args.gemv_q80_pro)
        if args.gemv_q80_slab is not None:
            rb.set_option(ttship.OPT["GEMV_Q80_SLAB"], args.gemv_q80_slab)
        if args.gemv_q80_rw is not None:
            rb.set_option(ttship.OPT["GEMV_Q80_RW"], args.gemv_q80_rw)
        if args.gemm_q8_staged is not None:
            rb.set_option(ttship.OPT["GEMM_Q8_STAGED"], args.gemm_q8_staged)
        if args.gemv_kr_inkernel is not None:
            rb.set_option(ttship.OPT["GEMV_KR_INKERNEL"], args.gemv_kr_inkernel)
        if args.attn_ks is not None:
            rb.set_option(ttship.OPT["ATTN_KS"], args.attn_ks)
        if args.attn_pv8 is not None:
            rb.set_option(ttship.OPT["ATTN_PV8"], args.attn_pv8)
        if args.kv_prefetch_blocks is not None:
            rb.set_option(ttship.OPT["KV_PREFETCH_BLOCKS"], args.kv_prefetch_blocks)
        return rb

    dcfg = ttship.dac_config(max_frames=args.steps)

    def new_dac(rb):
        if args.dac_conv_split is not None:  # concurrent decoders each sizing split convs for the whole chip
            rb.set_option(ttship.OPT["CONV_SPLIT"], args.dac_conv_split)
        rd = ttship.Dac(rb.iface(), dcfg)
        rd.decode(np.zeros((min(8, args.steps), dcfg.n_codebooks), dtype=np.int32))  # warm (code objects, arena)
        return rd

    reps = []
    for r in range(R):
        # a replica = one backend (its own HIP stream) + its own runners, as a server worker owns its
        # runners (examples/server/server.cpp:316-321); replicas run concurrently from host threads
        rb = new_backend()
        if args.cu_partition and R > 1:
            rb.set_option(ttship.OPT["CU_PARTITION"], (r << 8) | R | ((args.cu_partition - 1) << 16))
        rr = ttship.Parler(rb.iface(), cfg)
        rd = None if args.no_dac else new_dac(rb)
        reps.append((rb, rr, rd))
    be, runner, dac = reps[0]
    # DAC workers: the replicas' decoders plus extra backends of their own
    W = 0 if args.no_dac else max(1, min(args.dac_workers, args.batch))
    dac_workers = [(rb, rd) for rb, _, rd in reps[:W]]
    while len(dac_workers) < W:
        xb = new_backend()
        dac_workers.append((xb, new_dac(xb)))
    # text-prompt pass to reach the measured KV length (timed on its own: the prompt prefill, batch x ctx
    # columns per Q4_K product, on the matrix-core GEMM; not part of the headline's timed region)
    prefill_ms = []
    for r, (rb, rr, rd) in enumerate(reps):
        rb.sync()
        tp0 = time.perf_counter()
        rr.prefill(prompt_tokens(bl, args.ctx, cfg.prompt_vocab, offset=rank * args.batch + r * bl))
        rb.sync()
        prefill_ms.append(1000.0 * (time.perf_counter() - tp0))
        rr.generate(args.warmup)
        rb.sync()
    barrier_sync(dist, be)

    runner.host_stats(reset=True)
    c0 = be.counters()
    toks_r = [None] * R

    def ar_leg(r):
        rb, rr, _ = reps[r]
        toks_r[r] = rr.generate(args.steps)
        rb.sync()

    pcm = [None] * args.batch

    def dac_leg(w):
        # worker w decodes every W-th prompt of the whole per-GPU batch
        xb, rd = dac_workers[w]
        for g in range(w, args.batch, W):
            pcm[g] = rd.decode(dac_codes(toks_r[g // bl][g % bl], dcfg.codebook_size))
        xb.sync()

    t0 = time.perf_counter()
    run_replicas(ar_leg, R)
    t1 = time.perf_counter()
    c1 = be.counters()
    cdelta = {k: (c1.get(k, 0) - c0.get(k, 0)) / 1e3 / max(1, args.steps) for k in ("plan_wait_ns", "cap_plan_ns", "cap_launch_ns", "cap_update_ns")}
    if dac is not None:
        run_replicas(dac_leg, W)
    barrier_sync(dist, be)
    t2 = time.perf_counter()
    toks = np.concatenate(toks_r, axis=0)
    host = runner.host_stats(reset=True)
    # parts of compute_enqueue: waiting on the device for the plan slot, planner, launches under
    # capture (incl. planner), exec update
    host.update({k.replace("_ns", "_us"): round(v, 1) for k, v in cdelta.items()})
    b1 = None
    if args.b1_replicas > 0:
        barrier_sync(dist, be)
        b1 = parler_b1_leg(args, rank, local, new_backend)
        t = max_over_ranks(dist, local, b1["ms_per_step"])
        b1["ms_per_step"] = t
        b1["ar_audio_sec_per_s"] = round(world * args.b1_replicas * SAMPLES_PER_STEP / SAMPLE_RATE * 1000.0 / t, 3)
    kres = None
    if args.kokoro_prompts > 0:
        barrier_sync(dist, be)
        kres = kokoro_leg([rb for rb, _, _ in reps], args, rank, dist, local, world)
    ores = None
    if args.orpheus_steps > 0:
        barrier_sync(dist, be)
        ores = orpheus_leg(be, args, rank)
        # whole-job rate: every rank decoded its own shard; the slowest rank's step time sets it
        t = max_over_ranks(dist, local, ores["ms_per_step"])
        ores["ms_per_step"] = t
        ores["tokens_per_s"] = round(world * args.orpheus_batch * 1000.0 / t, 1)
        ores["audio_sec_per_s"] = round(ores["tokens_per_s"] / ORPHEUS_TOK_PER_AUDIO_S, 3)
    dres = None
    if args.dia_steps > 0:
        barrier_sync(dist, be)
        dres = dia_leg(be, args)
        t = max_over_ranks(dist, local, dres["ms_per_step"])
        dres["ms_per_step"] = t
        dres["audio_sec_per_s"] = round(world * SAMPLES_PER_STEP / SAMPLE_RATE * 1000.0 / t, 3)
    dt = max_over_ranks(dist, local, t2 - t0)
    dt_ar = max_over_ranks(dist, local, t1 - t0)
    dt_dac = max_over_ranks(dist, local, t2 - t1)
    gather_tokens(dist, rank, world, local, toks)
    # the one data exchange of the sharded job: every prompt's audio to rank 0
    gathered = None
    if dac is not None:
        tg0 = time.perf_counter()
        gathered = gather_audio(dist, rank, world, local, pcm)
        t_gather = time.perf_counter() - tg0

    total_prompts = args.batch * world
    audio_s = total_prompts * args.steps * SAMPLES_PER_STEP / SAMPLE_RATE
    roof = gemv_roofline(be, runner, max(5, min(40, args.steps // 5)))

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            ncpu = min(16, len(os.sched_getaffinity(0)))
            cpu = cpu_baseline(args, ncpu)
        what = "AR decode + DAC decode" if dac is not None else "AR decode"
        result = {
            "metric": f"audio-sec/wall-sec (RTF^-1), Parler-TTS-mini v1 Q4_K {what}",
            "value": round(audio_s / dt, 3),
            "unit": "audio-sec/wall-sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "q4_K weights x q8_K activations (int dot, f32 combine); DAC f16 im2col x f32 weights, f64 accumulate",
            "data": "synthetic (deterministic weights in Parler-mini v1 Q4_K and DAC-44k shapes; token ids from Harvard sentences)",
            "config": {"workload": f"Parler-TTS-mini-v1 Q4_K, greedy AR decode + DAC-44k (BASELINE configs[2])",
                       "model": "parler-tts-mini-v1", "prompts_per_gpu": args.batch, "global_batch": total_prompts,
                       "kv_len_start": args.ctx, "frames_per_prompt": args.steps,
                       "parallelism": f"dp{world} (prompt shards), {R} concurrent replicas x {bl} prompts per GPU, {W} concurrent DAC decoders",
                       "graph_nodes_per_step": runner.last_graph_nodes(),
                       "dac_graph_nodes": dac.last_graph_nodes() if dac is not None else None},
            "ar_audio_sec_per_s": round(audio_s / dt_ar, 3),
            "ar_ms_per_step": round(1000.0 * dt_ar / args.steps, 4),
            "dac_audio_sec_per_s": round(audio_s / dt_dac, 3) if dac is not None else None,
            "codec_tokens_per_s": round(total_prompts * args.steps * HEADS / dt_ar, 1),
            "host_us_per_step": host,
            "prefill_ms": {"per_replica": [round(v, 2) for v in prefill_ms], "prompts": bl, "tokens_per_prompt": args.ctx,
                           "note": "prompt pass to the KV start length (untimed by the headline)"},
            "audio_gather": None if gathered is None else {
                "prompts": len(gathered), "audio_sec": round(sum(len(p) for p in gathered) / SAMPLE_RATE, 3),
                "ms": round(1000.0 * t_gather, 3), "transport": "RCCL send/recv (gatherv) to rank 0" if world > 1 else "local"},
            "parler_b1": b1,
            "kokoro": kres,
            "orpheus": ores,
            "dia": dres,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    for xb, rd in dac_workers[R:]:
        rd.close()
        xb.close()
    for rb, rr, rd in reps:
        if rd is not None:
            rd.close()
        rr.close()
        rb.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
