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
# PMC traffic of the Dia leg's slab Q8_0 GEMV (scripts/gpu_pmc_r6.sh)
PMC_FILE_DIA = max((ROOT / "profiles").glob("r*/pmc_gemv_q8_0s_dia.json"), default=None)
# PMC traffic of the decode attention pair at the headline's KV length (scripts/gpu_pmc_r6.sh)
PMC_FILE_ATTN = max((ROOT / "profiles").glob("r*/pmc_attn_kv448.json"), default=None)

# examples/perf_battery/perf_battery.cpp:25-56: the reference's 29 test prompts (its list has 30 literals, but
# "Kick the ball straight and follow through." lacks a comma, so C++ joins it with the next one)
HARVARD = [
    "The birch canoe slid on the smooth planks.",
    "Glue the sheet to the dark blue background.",
    "It's easy to tell the depth of a well.",
    "These days a chicken leg is a rare dish.",
    "Rice is often served in round bowls.",
    "The juice of lemons makes fine punch.",
    "The box was thrown beside the parked truck.",
    "The hogs were fed chopped corn and garbage.",
    "Four hours of steady work faced us.",
    "A large size in stockings is hard to sell.",
    "The boy was there when the sun rose.",
    "A rod is used to catch pink salmon.",
    "The source of the huge river is the clear spring.",
    "Kick the ball straight and follow through.Help the woman get back to her feet.",
    "A pot of tea helps to pass the evening.",
    "Smoky fires lack flame and heat.",
    "The soft cushion broke the man's fall.",
    "The salt breeze came across from the sea.",
    "The girl at the booth sold fifty bonds.",
    "The small pup gnawed a hole in the sock.",
    "The fish twisted and turned on the bent hook.",
    "Press the pants and sew a button on the vest.",
    "The swan dive was far short of perfect.",
    "The beauty of the view stunned the young boy.",
    "Two blue fish swam in the tank.",
    "Her purse was full of useless trash.",
    "The colt reared and threw the tall rider.",
    "It snowed, rained, and hailed the same morning.",
    "Read verse out loud for pleasure.",
]


def sentence_tokens(s, vocab):
    """Stand-in for the T5 ids of one prompt (the tokenizer model is not available offline): one id per word
    piece (words and punctuation) plus the closing </s> (id 1), so a prompt pass has the sentence's length."""
    import re
    pieces = re.findall(r"[A-Za-z']+|[^\sA-Za-z']", s)
    return np.asarray([(sum(p.encode()) * 131 + len(p) * 7) % (vocab - 2) + 2 for p in pieces] + [1], dtype=np.int32)


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


def cpu_baseline(args, n_threads, B):
    """Oracle (C restatement of ggml-cpu) on the GPU leg's workload shape, on host cores: the same
    Parler step graph at the same lock-step batch as one GPU replica and the same KV length when timing
    starts (tts_parler_set_position: the prefill is skipped, the step's work is the same), then the
    same DAC graph over a few frames per prompt; rates per audio-second, end to end = 1 / (1/AR + 1/DAC)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import py_oracle
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
    frames, nd = 2, min(B, 8)
    dcfg = ttship.dac_config(max_frames=frames)
    dac = ttship.Dac(py_oracle.iface(n_threads), dcfg)
    try:
        t0 = time.perf_counter()
        for b in range(nd):
            dac.decode(dac_codes(toks[b], dcfg.codebook_size))
        dt_dac = time.perf_counter() - t0
    finally:
        dac.close()
    ar = B * steps * SAMPLES_PER_STEP / SAMPLE_RATE / dt_ar
    dac_rate = nd * frames * SAMPLES_PER_STEP / SAMPLE_RATE / dt_dac
    return {"value": 1.0 / (1.0 / ar + 1.0 / dac_rate), "unit": "audio-sec/wall-sec", "cores": n_threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "sample": f"{steps} Parler-mini Q4_K decode steps of {B} lock-step prompts (one GPU replica's batch) at KV length "
                      f"{args.ctx} (prefill skipped) + DAC-44k decode of {frames} frames for {nd} prompts (oracle/ggml_ref.c, C "
                      f"restatement of ggml-cpu scalar paths, {n_threads} threads = the box's CPU share; reference ggml-cpu "
                      f"unbuildable offline)",
            "ar_audio_sec_per_s": round(ar, 5), "dac_audio_sec_per_s": round(dac_rate, 5),
            "codec_tokens_per_s": B * steps * HEADS / dt_ar}


F64_MFMA_PEAK_TF = 47.0  # measured v_mfma_f64_16x16x4f64 rate on the box (scripts/mfma_f64_peak.hip)


def dac_flops_per_frame(dcfg):
    """Algorithmic FLOPs of the DAC-44k decoder per codec frame (2 x multiply-adds of the reference's
    convs, general_neural_audio_codec.cpp:133-172 / dac_model.cpp:139-170): the quantizer out-projections,
    the initial k7 conv, per layer the conv_transpose_1d (kernel 2 x rate, stride rate: 2 x Cin x Cout per
    output sample) and three residual units (k7 + k1 convs), the final k7 conv to one channel."""
    rates = list(dcfg.rates)[:dcfg.n_layers]
    macs = dcfg.n_codebooks * dcfg.codebook_dim * dcfg.latent_dim + 7 * dcfg.latent_dim * dcfg.decoder_dim
    c, s = dcfg.decoder_dim, 1
    for r in rates:
        co = c // 2
        s *= r
        macs += 2 * c * co * s + 3 * (7 + 1) * co * co * s
        c = co
    macs += 7 * c * s
    return 2 * macs


def copy_peak(be, nbytes=1 << 30, reps=10):
    """The measured HBM ceiling beside the 8 TB/s spec: a streaming copy kernel
    (tts_hip_copy_stream: 16-B non-temporal loads / stores per lane, one contiguous chunk per workgroup, the
    guide's float4-copy method) of
    `nbytes` on the backend's stream, read + write bytes per second over `reps` copies after one warm
    copy; and the runtime's device-to-device copy (tts_hip_tensor_copy) the same way."""
    L = ttship.lib()
    a, b = be.alloc(nbytes), be.alloc(nbytes)
    out = {}
    try:
        for name, fn in (("kernel", L.tts_hip_copy_stream), ("runtime", L.tts_hip_tensor_copy)):
            if fn(be.ptr, b, a, nbytes) != 0:
                raise RuntimeError(f"{name} copy failed")
            be.sync()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn(be.ptr, b, a, nbytes)
            be.sync()
            out[name] = round(2.0 * nbytes * reps / (time.perf_counter() - t0) / 1e9, 1)
    finally:
        be.free(a)
        be.free(b)
    return out


def gemv_roofline(be, runner, steps):
    """Dominant kernels of the decode step, from HIP events carried in their dispatch packets over
    profiled steps: the Q4_K dequant-GEMV / matrix-core GEMM launches (algorithmic bytes per launch =
    every weight byte once + activations + outputs) and the decode attention's scores + P.V pair
    (bytes = every K and V row read).  `traffic` is PMC HBM bytes per launch from a committed
    rocprofv3 pass (source and mode named beside it), not taken in this run."""
    be.set_option(1, 1)
    be.gemv_stats(-1, reset=True)
    runner.generate(steps)
    ms, launches, nbytes = be.gemv_stats(ttship.Q4_K, reset=False)
    ams, alaunches, abytes = be.gemv_stats(ttship.PROF_ATTN, reset=True)
    be.set_option(1, 0)
    avg_us = 1000.0 * ms / max(launches, 1)
    bpl = nbytes / max(launches, 1)
    gbs = bpl / (avg_us * 1e-6) / 1e9 if launches else 0.0
    traffic, src, mode = None, None, None
    if PMC_FILE.exists():
        pmc = json.loads(PMC_FILE.read_text())
        traffic, src, mode = pmc.get("hbm_bytes_per_launch"), str(PMC_FILE.relative_to(ROOT)), pmc.get("command")
    pa = json.loads(PMC_FILE_ATTN.read_text()) if PMC_FILE_ATTN else {}
    a_us = 1000.0 * ams / max(alaunches, 1)
    a_bpl = abytes / max(alaunches, 1)
    a_gbs = a_bpl / (a_us * 1e-6) / 1e9 if alaunches else 0.0
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src, "traffic_mode": mode,
            "kernel": "k_gemv_q4K_kr (K-relay matrix-core GEMM, > 8 lock-step columns) / k_gemv_q4_K (<= 8)",
            "avg_launch_us": round(avg_us, 3), "bytes_per_launch": round(bpl, 1), "launches_sampled": launches,
            "attention": {"kernel": "k_attn_scores + k_attn_pv (one decode attention)", "achieved": round(a_gbs, 1),
                          "frac": round(a_gbs / HBM_PEAK_GBS, 4), "avg_us": round(a_us, 3), "bytes_per_call": round(a_bpl, 1),
                          "calls_sampled": alaunches, "traffic": pa.get("pair_hbm_bytes_per_call"),
                          "traffic_source": str(PMC_FILE_ATTN.relative_to(ROOT)) if PMC_FILE_ATTN else None}}


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


ORPHEUS_HEADS = (0, 1, 2, 2, 1, 2, 2)  # SNAC codebook of each token in a 7-token frame (orpheus model.h heads)


def orpheus_snac_heads(toks):
    """orpheus_runner::prepare_output_tokens (src/models/orpheus/model.cpp:370-386): whole 7-token
    frames, token ii of a frame -> codebook heads[ii], code = token - 128266 - ii * 4096.  Synthetic
    weights emit arbitrary ids, so codes are folded into [0, 4096) (a trained model emits in range)."""
    n = len(toks) // 7 * 7
    heads = [[], [], []]
    for i in range(n):
        ii = i % 7
        heads[ORPHEUS_HEADS[ii]].append((int(toks[i]) - 128266 - ii * 4096) % 4096)
    return [np.asarray(h, dtype=np.int32) for h in heads]


def orpheus_leg(be, args, rank):
    """BASELINE configs[4] per-GPU shard: Orpheus-3B Q4_K (synthetic weights, every matrix incl. the
    156 940-row head in Q4_K), `orpheus_batch` prompts in lockstep, greedy decode with device
    sampling, then every prompt's tokens through the SNAC-24k vocoder (orpheus model.cpp:389-405:
    prepare_output_tokens + snac_runner::run) -- audio_sec_per_s counts produced PCM over decode + SNAC;
    plus the dequant-GEMV roofline over profiled steps."""
    B, steps, n_prompt = args.orpheus_batch, args.orpheus_steps, 32
    cfg = ttship.orpheus_config(batch=B, max_ctx=n_prompt + steps + 64, arena_bytes=1 << 30)
    o = ttship.Orpheus(be.iface(), cfg)
    scfg = ttship.snac_config(max_frames=4 * (steps // 7) + 8)
    snac = ttship.Snac(be.iface(), scfg)
    try:
        prompt = (np.arange(B * n_prompt, dtype=np.int32).reshape(B, n_prompt) * 7919 + 128000 + rank) % cfg.vocab_size
        first = o.prefill(prompt).argmax(axis=1).astype(np.int32)
        toks = o.generate(first, 4)
        heads0 = orpheus_snac_heads((toks[0].tolist() * 7)[:7])  # one 7-token frame
        snac.decode(heads0, np.zeros(snac.noise_per_frame * len(heads0[-1]), np.float32))  # warm
        rng = np.random.default_rng(rank)
        be.sync()
        t0 = time.perf_counter()
        toks = o.generate(toks[:, -1], steps)
        be.sync()
        t1 = time.perf_counter()
        samples = 0
        for b in range(B):
            hs = orpheus_snac_heads(toks[b])
            noise = rng.standard_normal(snac.noise_per_frame * len(hs[-1])).astype(np.float32)
            samples += snac.decode(hs, noise).shape[0]
        be.sync()
        t2 = time.perf_counter()
        dt = t1 - t0
        be.set_option(ttship.OPT["PROFILE_GEMV"], 1)
        be.gemv_stats(-1, reset=True)
        o.generate(toks[:, -1], 8)
        ms, launches, nbytes = be.gemv_stats(ttship.Q4_K, reset=True)
        be.set_option(ttship.OPT["PROFILE_GEMV"], 0)
        avg_us = 1000.0 * ms / max(launches, 1)
        gbs = nbytes / max(launches, 1) / (avg_us * 1e-6) / 1e9 if launches else 0.0
        pmc = json.loads(PMC_FILE_ORPH.read_text()) if PMC_FILE_ORPH else {}
        return {"workload": f"Orpheus-3B Q4_K greedy decode (BASELINE configs[4] per-GPU shard), {B} prompts, prompt {n_prompt} + "
                            f"{steps} timed steps, then SNAC-24k of every prompt's {steps // 7} frames; synthetic weights",
                "tokens_per_s": round(B * steps / dt, 1), "ms_per_step": round(1000 * dt / steps, 3),
                "snac_ms": round(1000 * (t2 - t1), 3), "audio_sec_per_gpu": round(samples / 24000.0, 4), "wall_s": t2 - t0,
                "audio_sec_per_s": round(samples / 24000.0 / (t2 - t0), 3),
                "graph_nodes": o.last_graph_nodes(), "weight_bytes": o.weight_bytes(),
                "roofline": {"bound": "hbm", "kernel": "k_gemv_q4K_kr (K relay, tile layout, >= 4 MiB; its operand pass k_quant_mf "
                                                      "not included) + k_gemv_q4_K (k / v lane layout)",
                             "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "avg_launch_us": round(avg_us, 3), "bytes_per_launch": round(nbytes / max(launches, 1), 1),
                             "launches_sampled": launches, "traffic_kr": pmc.get("hbm_bytes_per_launch"),
                             "traffic_source": str(PMC_FILE_ORPH.relative_to(ROOT)) if PMC_FILE_ORPH else None,
                             "traffic_mode": pmc.get("command")}}
    finally:
        snac.close()
        o.close()


DIA_DELAYS = (0, 8, 9, 10, 11, 12, 13, 14, 15)  # Dia's delay pattern (dia model.h), max_delay 15


def dia_frames(toks):
    """dia_runner::adjust_output_tokens (src/models/dia/model.cpp:825-846): frame i takes head ii's token
    of step i + delay[ii]; synthetic weights' ids >= 1024 (BOS / EOS / pad) are folded into the codebook
    range instead of dropping the frame, so every step yields audio."""
    n = toks.shape[0] - DIA_DELAYS[-1]
    return np.stack([toks[i + np.array(DIA_DELAYS), np.arange(9)] % 1024 for i in range(n)]).astype(np.int32)


def dialogue(n_chars):
    """A two-speaker dialogue (Dia's [S1] / [S2] speaker tags as the tokenizer's bytes 0x01 / 0x02) of
    Harvard sentences, cut to n_chars bytes (tests/test_dia_gpu.py)."""
    out, i = b"", 0
    while len(out) < n_chars:
        out += (b"\x01 " if i % 2 == 0 else b" \x02 ") + HARVARD[i % len(HARVARD)].encode()
        i += 1
    return np.frombuffer(out[:n_chars], dtype=np.uint8).astype(np.int32)


def dia_leg(be, args):
    """BASELINE configs[3]: Dia-1.6B Q8_0 (synthetic weights), the encoder step over a long-form
    two-speaker dialogue (the whole 1024-position encoder context), timed CFG decoder steps (conditioned
    + unconditioned in one graph, greedy heads fed back), then the delay pattern undone and the frames
    through DAC-44k (dia model.cpp:849-870); audio_sec_per_s counts produced PCM over decode + DAC.
    Plus the Q8_0 slab GEMV roofline over profiled steps."""
    dcfg = ttship.dia_config(max_generation_size=args.dia_steps + 16)
    d = ttship.Dia(be.iface(), dcfg)
    dac = ttship.Dac(be.iface(), ttship.dac_config(max_frames=args.dia_steps))
    try:
        text = dialogue(dcfg.max_encoder_context_length)
        t0 = time.perf_counter()
        audio = d.prefill(text, np.full(9, 1026, dtype=np.int32)).argmax(axis=1).astype(np.int32)
        t_enc = time.perf_counter() - t0
        audio = d.generate(audio, 3)[-1]  # warm (plans, code objects)
        dac.decode(np.zeros((8, 9), np.int32))
        be.sync()
        t0 = time.perf_counter()
        toks = d.generate(audio, args.dia_steps)  # device-resident greedy loop
        be.sync()
        t1 = time.perf_counter()
        pcm = dac.decode(dia_frames(toks))
        be.sync()
        t2 = time.perf_counter()
        dt = t1 - t0
        be.set_option(ttship.OPT["PROFILE_GEMV"], 1)
        be.gemv_stats(-1, reset=True)
        d.generate(toks[-1], 8)
        ms, launches, nbytes = be.gemv_stats(ttship.Q8_0, reset=True)
        be.set_option(ttship.OPT["PROFILE_GEMV"], 0)
        pmc = json.loads(PMC_FILE_DIA.read_text()) if PMC_FILE_DIA else {}
        avg_us = 1000.0 * ms / max(launches, 1)
        gbs = nbytes / max(launches, 1) / (avg_us * 1e-6) / 1e9 if launches else 0.0
        return {"workload": f"Dia-1.6B Q8_0 CFG decode (BASELINE configs[3]), 1 prompt = a {len(text)}-byte two-speaker dialogue, "
                            f"{args.dia_steps} timed steps, then DAC-44k of the {args.dia_steps - DIA_DELAYS[-1]} undelayed frames; "
                            "synthetic weights",
                "ms_per_step": round(1000 * dt / args.dia_steps, 3), "dac_ms": round(1000 * (t2 - t1), 3),
                "ar_audio_sec_per_s": round(args.dia_steps * SAMPLES_PER_STEP / SAMPLE_RATE / dt, 3),
                "audio_sec_per_gpu": round(pcm.shape[0] / SAMPLE_RATE, 4), "wall_s": t2 - t0,
                "audio_sec_per_s": round(pcm.shape[0] / SAMPLE_RATE / (t2 - t0), 3),
                "encoder_step_ms": round(1000 * t_enc, 1), "weight_bytes": d.weight_bytes(),
                "roofline": {"bound": "hbm", "kernel": "k_gemv_q8_0s (slab Q8_0 GEMV, <= 8 columns)", "achieved": round(gbs, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_launch_us": round(avg_us, 3),
                             "bytes_per_launch": round(nbytes / max(launches, 1), 1), "launches_sampled": launches,
                             "traffic": pmc.get("hbm_bytes_per_launch"),
                             "traffic_source": str(PMC_FILE_DIA.relative_to(ROOT)) if PMC_FILE_DIA else None,
                             "traffic_mode": pmc.get("command")}}
    finally:
        dac.close()
        d.close()


def parler_b1_leg(args, rank, local, new_backend, R=None, coalesce=True, ragged=False):
    """TTS.cpp's serving shape (examples/server/server.cpp:316-321,885-895): one prompt per runner, R
    runners, each on its own backend (HIP stream) with its own model copy, driven by its own host thread
    through TTS.cpp's own step loop (graph_compute, logits read back, host greedy sampler:
    parler_tts_runner::decode, src/models/parler/model.cpp:648-693).
    coalesce=True: the backend's step coalescer (coalesce.hip) runs the runners' steps as batched
    launches; False: every runner alone (TTS_HIP_OPT_COALESCE = 0).  ragged=False: every runner prefilled
    to the same KV length, started together; True: runner r's prompt is 7 r tokens longer and its thread
    starts r ms later (the server's requests arrive at different times with different lengths)."""
    R, steps = R or args.b1_replicas, args.b1_steps
    # the same KV capacity rule as the lock-step leg: a multiple of 4 positions keeps every V row
    # 16-B aligned, so P.V takes its vector-load kernel (k_attn_pv<true, ...>)
    cfg = ttship.parler_config(batch=1, max_ctx=max(4096, args.ctx + 7 * R + steps + args.warmup + 64))
    bes = [new_backend() for _ in range(R)]
    for b in bes:
        b.set_option(ttship.OPT["COALESCE"], 1 if coalesce else 0)
    runs = [None] * R
    lens = [args.ctx + (7 * r if ragged else 0) for r in range(R)]

    def make(r):  # each worker loads its own model copy (runner_from_file per worker, server.cpp:316-321)
        runs[r] = ttship.Parler(bes[r].iface(reference_flow=True), cfg)
        runs[r].prefill(prompt_tokens(1, lens[r], cfg.prompt_vocab, offset=rank * R + r))
        bes[r].sync()

    try:
        run_replicas(make, R)
        run_replicas(lambda r: (runs[r].generate(args.warmup), bes[r].sync()), R)  # the coalesced groups form
        s0 = ttship.coalesce_stats(local)
        runs[0].host_stats(reset=True)

        def one(r):
            if ragged:
                time.sleep(0.001 * r)
            runs[r].generate(steps)
            bes[r].sync()

        t0 = time.perf_counter()
        run_replicas(one, R)
        dt = time.perf_counter() - t0
        s1 = ttship.coalesce_stats(local)
        co = {k: s1[k] - s0[k] for k in ("launches", "member_steps", "alone", "refused", "ragged_launches")}
        co["max_group"] = s1["max_group"]
        co["wait_us_per_step"] = round((s1["wait_us"] - s0["wait_us"]) / max(1, R * steps), 1)
        co["runner0_host_us_per_step"] = runs[0].host_stats(reset=True)  # build / alloc / set_inputs / compute (incl. the rendezvous) / get
        nl = max(1, co["launches"])  # host time per coalesced launch: the whole run_group, its layout / plan / tables parts
        co["host_us_per_launch"] = {k: round((s1[k] - s0[k]) / nl, 1) for k in ("exec_us", "layout_us", "plan_us", "tables_us")}
        return {"workload": f"Parler-mini Q4_K AR decode, {R} runners x 1 prompt (TTS.cpp's server model: one runner, backend and "
                            f"model copy per worker thread, graph_compute + host greedy sampler per step), KV "
                            f"{min(lens)}..{max(lens)} -> +{steps}" + (", prompt lengths 7 r apart, thread r starting r ms late" if ragged else ""),
                "replicas": R, "batch_per_replica": 1,
                "step_coalescer": "on" if coalesce else "off", "coalescer": co,
                "ms_per_step": round(1000 * dt / steps, 4),
                "ar_audio_sec_per_s": round(R * steps * SAMPLES_PER_STEP / SAMPLE_RATE / dt, 3)}
    finally:
        for p in runs:
            if p is not None:
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


def parler_replicas(args, per_gpu, R, rank, new_backend, dac_cfg=None):
    """R replicas (each its own backend = HIP stream, driven by its own host thread) of per_gpu / R
    lock-step prompts, prefilled to the KV start length and warmed; + per-replica prefill times."""
    bl = per_gpu // R
    # the compute arena holds the prompt pass too (attention scores [ctx, ctx, H, prompts]): 4 GiB per 8 prompts
    cfg = ttship.parler_config(batch=bl, max_ctx=max(4096, args.ctx + args.steps + args.warmup + 64),
                               arena_bytes=max(4, (bl + 7) // 8 * 4) << 30)
    reps, prefill_ms = [], []
    for r in range(R):
        rb = new_backend()
        if args.cu_partition and R > 1:
            rb.set_option(ttship.OPT["CU_PARTITION"], (r << 8) | R | ((args.cu_partition - 1) << 16))
        rr = ttship.Parler(rb.iface(), cfg)
        rd = None if dac_cfg is None else new_dac_for(args, rb, dac_cfg)
        reps.append((rb, rr, rd))
    for r, (rb, rr, rd) in enumerate(reps):
        rb.sync()
        tp0 = time.perf_counter()
        if getattr(args, "no_prefill", False):  # (counter runs: the decode step's work at KV ctx without the long prompt pass)
            rr.prefill(prompt_tokens(bl, 8, cfg.prompt_vocab, offset=rank * per_gpu + r * bl))
            rr.set_position(args.ctx)
        else:
            rr.prefill(prompt_tokens(bl, args.ctx, cfg.prompt_vocab, offset=rank * per_gpu + r * bl))
        rb.sync()
        prefill_ms.append(1000.0 * (time.perf_counter() - tp0))
        rr.generate(min(2, args.warmup))  # the step graph recorded (first sighting eager, then captured)
        rb.sync()
    return reps, prefill_ms, cfg


def warm_concurrent(args, reps):
    """The rest of the W warmup steps with every replica running at once, right before the timed
    region: the device sees the timed shape (and its clocks) immediately before timing starts, whatever
    ran before it (DAC workers' setup, another leg)."""
    n = max(0, args.warmup - min(2, args.warmup))
    if n:
        run_replicas(lambda r: (reps[r][1].generate(n), reps[r][0].sync()), len(reps))


def new_dac_for(args, rb, dcfg):
    if args.dac_conv_split is not None:  # concurrent decoders each sizing split convs for the whole chip
        rb.set_option(ttship.OPT["CONV_SPLIT"], args.dac_conv_split)
    rd = ttship.Dac(rb.iface(), dcfg)
    nbd = dac_batch(args)
    if nbd > 1:  # warm the batched shape twice: the first sighting launches eagerly, the second records the graph
        for _ in range(2):
            rd.decode_batch(np.zeros((nbd, args.steps, dcfg.n_codebooks), dtype=np.int32))
    else:
        rd.decode(np.zeros((min(8, args.steps), dcfg.n_codebooks), dtype=np.int32))  # warm (code objects, arena)
    return rd


def dac_batch(args):
    """Prompts per batched DAC decode: short codec sequences fill few CUs, so up to 64 frames per prompt
    several prompts decode as one graph (tts_dac_decode_batch) -- 8, or half the GPU's prompts when it
    has fewer than 16, so two decoders still overlap (measured: 64 prompts 8 x 8 best, 8 prompts 2 x 4
    best); longer sequences one by one (861 frames: 1, 2 and 4 per decode within 1 %)."""
    if args.dac_batch is not None:
        return max(1, args.dac_batch)
    if args.steps > 64:
        return 1
    return min(8, max(1, getattr(args, "per_gpu_", 64) // 2))


def close_replicas(reps):
    for rb, rr, rd in reps:
        if rd is not None:
            rd.close()
        rr.close()
        rb.close()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=861, help="AR steps per prompt (861 = 10.0 s of audio, SURVEY §8d)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prompts", type=int, default=64, help="the fixed synthetic prompt set (north_star: a 64-prompt batch), "
                    "split over the ranks: strong scaling")
    ap.add_argument("--batch", type=int, default=None, help="prompts per GPU instead of --prompts / world (weak scaling)")
    ap.add_argument("--ctx", type=int, default=448, help="KV length when timing starts (prompt prefill)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prefill", action="store_true", help="counter / trace runs: an 8-token prompt pass, then the KV length "
                    "set to --ctx (tts_parler_set_position: the decode steps do the work of KV ctx without its prompt pass)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-steps", type=int, default=400)
    ap.add_argument("--b1-replicas", type=int, default=8, help="the B=1 leg: this many runners of one prompt each, as "
                    "TTS.cpp's server workers run (0 = skip)")
    ap.add_argument("--b1-steps", type=int, default=100)
    ap.add_argument("--b1-wide", type=int, default=32, help="the ragged B=1 leg again with this many coalesced runners (0 = skip)")
    ap.add_argument("--b1-coalesce", type=int, default=1, help="1: also run the B=1 legs with the step coalescer (equal and "
                    "ragged KV lengths; 0 = only the runners alone)")
    ap.add_argument("--sampled-steps", type=int, default=20, help="the headline's AR decode again with seeded top-k 50 sampling "
                    "(the reference's default sampler) for this many steps (0 = skip)")
    ap.add_argument("--prompt-pass", type=int, default=1, help="time every prompt's own sentence prompt pass from position 0 (0 = skip)")
    ap.add_argument("--p8", type=int, default=1, help="beside the headline, the AR line at 8 prompts per GPU (2 replicas x 4: "
                    "the 64-prompt batch over 8 GPUs) when the headline runs more (0 = skip)")
    ap.add_argument("--no-fusion", action="store_true")
    ap.add_argument("--fusion-mask", type=int, default=None, help="TTS_HIP_OPT_FUSION: TTS_FUSE_* bitmask (default: all)")
    ap.add_argument("--no-dac", action="store_true", help="AR decode only")
    ap.add_argument("--attn-split", type=int, default=None, help="TTS_HIP_OPT_ATTN_SPLIT: min KV length for split attention (0 = off)")
    ap.add_argument("--replicas", type=int, default=2, help="concurrent runner replicas per GPU, each on its own "
                    "backend/stream with prompts/replicas lock-step prompts (the server's worker model)")
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
    ap.add_argument("--attn-pv-mp", type=int, default=None, help="TTS_HIP_OPT_ATTN_PV_MP: all dims of a head per P.V workgroup (1) or 16 (0)")
    ap.add_argument("--gemm-kr-cp", type=int, default=None, help="TTS_HIP_OPT_GEMM_KR_CP: two column tiles per K-relay workgroup on parallel wave halves (1) or not (0)")
    ap.add_argument("--gemm-kr-walk", type=int, default=None, help="TTS_HIP_OPT_GEMM_KR_WALK: row-tile walkers per column tile of the prompt pass's many-column K-relay GEMM (0 = one workgroup per tile pair)")
    ap.add_argument("--gemm-pf", type=int, default=None, help="TTS_HIP_OPT_GEMM_PF: min columns of a Q4_K product on the prefill GEMM (0 = K-relay GEMM)")
    ap.add_argument("--gemm-kr-xcd", type=int, default=None, help="TTS_HIP_OPT_GEMM_KR_XCD: a row tile's column tiles on one XCD (1) or grid order (0, default)")
    ap.add_argument("--gemm-kr-nw", type=int, default=None, help="TTS_HIP_OPT_GEMM_KR_NW: waves per tile of the many-column K-relay GEMM (4 / 8)")
    ap.add_argument("--gemv-f32-wide", type=int, default=None, help="TTS_HIP_OPT_GEMV_F32_WIDE: wide GEMV for the F32 heads at 9..64 columns (1) or the tiled GEMM (0)")
    ap.add_argument("--graphs", type=int, default=1, help="replay each step as a HIP graph (1) or launch eagerly (0)")
    ap.add_argument("--cu-partition", type=int, default=0, help="TTS_HIP_OPT_CU_PARTITION for the AR replicas: 0 = every "
                    "replica on all CUs, 1 = replica r on the r-th contiguous CU set, 2 = on CUs c with c %% R == r")
    ap.add_argument("--dac-conv-split", type=int, default=None, help="TTS_HIP_OPT_CONV_SPLIT on the DAC workers' backends "
                    "(split convs over extra workgroups; default: the backend's default, on)")
    ap.add_argument("--dac-workers", type=int, default=8, help="concurrent DAC decoders per GPU (each its own backend / "
                    "stream; the AR replicas' backends first): short codec sequences fill few CUs, so several "
                    "prompts decode side by side")
    ap.add_argument("--dac-batch", type=int, default=None, help="prompts per batched DAC decode (tts_dac_decode_batch: one "
                    "graph, zeroed gaps, PCM bit-identical to one decode per prompt); default: 8 up to 64 frames, else 1")
    ap.add_argument("--idle-ms", type=float, default=0.0, help="study: idle host sleep between the warmup and the timed region")
    ap.add_argument("--kokoro-prompts", type=int, default=8, help="Kokoro-82M prompts per GPU, end to end (0 = skip)")
    ap.add_argument("--orpheus-steps", type=int, default=64, help="timed Orpheus-3B decode steps per GPU (0 = skip)")
    ap.add_argument("--orpheus-batch", type=int, default=8, help="Orpheus prompts per GPU (64-prompt batch / 8 GPUs)")
    ap.add_argument("--dia-steps", type=int, default=64, help="timed Dia-1.6B decoder steps per GPU (0 = skip)")
    args = ap.parse_args()

    rank, world, local, dist = dist_init()
    R = args.replicas
    strong = args.batch is None
    if strong and args.prompts % world:
        raise SystemExit(f"--prompts {args.prompts} must split evenly over {world} GPUs")
    per_gpu = args.prompts // world if strong else args.batch
    args.per_gpu_ = per_gpu  # (dac_batch)
    if R < 1 or per_gpu % R:
        raise SystemExit(f"--replicas {R} must divide the {per_gpu} prompts per GPU")
    bl = per_gpu // R  # prompts per replica

    def new_backend():
        rb = ttship.HipBackend(local)
        if args.no_fusion:
            rb.set_option(0, 0)
        elif args.fusion_mask is not None:
            rb.set_option(0, args.fusion_mask)
        rb.set_option(2, args.graphs)
        for flag, opt in (("conv_acc", "CONV_F32ACC"), ("attn_split", "ATTN_SPLIT"), ("kv_prefetch", "KV_PREFETCH"),
                          ("gemv_unique", "GEMV_UNIQUE"), ("tile_bytes", "Q4K_TILE_BYTES"), ("gemv_ks", "GEMV_KS"),
                          ("attn_fused", "ATTN_FUSED"), ("attn_pv16", "ATTN_PV16"), ("gemv_krelay", "GEMV_KRELAY"),
                          ("gemv_nw_min", "GEMV_NW_MIN"), ("gemv_q80_pro", "GEMV_Q80_PRO"), ("gemv_q80_slab", "GEMV_Q80_SLAB"),
                          ("gemv_q80_rw", "GEMV_Q80_RW"), ("gemm_q8_staged", "GEMM_Q8_STAGED"),
                          ("gemv_kr_inkernel", "GEMV_KR_INKERNEL"), ("attn_ks", "ATTN_KS"), ("attn_pv8", "ATTN_PV8"),
                          ("kv_prefetch_blocks", "KV_PREFETCH_BLOCKS"), ("gemv_f32_wide", "GEMV_F32_WIDE"),
                          ("attn_pv_mp", "ATTN_PV_MP"), ("gemm_kr_nw", "GEMM_KR_NW"), ("gemm_kr_xcd", "GEMM_KR_XCD"), ("gemm_kr_cp", "GEMM_KR_CP"), ("gemm_kr_walk", "GEMM_KR_WALK"), ("gemm_pf", "GEMM_PF")):
            v = getattr(args, flag)
            if v is not None:
                rb.set_option(ttship.OPT[opt], v)
        return rb

    # (batched decodes: nb prompts + the gaps between them, <= 8 frames each, in one graph)
    dcfg = ttship.dac_config(max_frames=args.steps if dac_batch(args) == 1 else dac_batch(args) * (args.steps + 8))
    reps, prefill_ms, cfg = parler_replicas(args, per_gpu, R, rank, new_backend, None if args.no_dac else dcfg)
    be, runner, dac = reps[0]
    # DAC workers: the replicas' decoders plus extra backends of their own
    NBD = min(dac_batch(args), per_gpu)
    n_dac_batches = (per_gpu + NBD - 1) // NBD
    W = 0 if args.no_dac else max(1, min(args.dac_workers, n_dac_batches))
    dac_workers = [(rb, rd) for rb, _, rd in reps[:W]]
    while len(dac_workers) < W:
        xb = new_backend()
        dac_workers.append((xb, new_dac_for(args, xb, dcfg)))
    warm_concurrent(args, reps)
    if args.idle_ms:  # study: an idle gap between the warmup and the timed region
        time.sleep(args.idle_ms / 1e3)
    barrier_sync(dist, be)

    runner.host_stats(reset=True)
    c0 = be.counters()
    toks_r = [None] * R

    def ar_leg(r):
        rb, rr, _ = reps[r]
        toks_r[r] = rr.generate(args.steps)
        rb.sync()

    pcm = [None] * per_gpu

    def dac_leg(w):
        # worker w decodes every W-th batch of NBD prompts of this GPU's prompts
        xb, rd = dac_workers[w]
        for bt in range(w, n_dac_batches, W):
            gs = list(range(bt * NBD, min(per_gpu, (bt + 1) * NBD)))
            if len(gs) == 1 or NBD == 1:
                for g in gs:
                    pcm[g] = rd.decode(dac_codes(toks_r[g // bl][g % bl], dcfg.codebook_size))
            else:
                out = rd.decode_batch(np.stack([dac_codes(toks_r[g // bl][g % bl], dcfg.codebook_size) for g in gs]))
                for i, g in enumerate(gs):
                    pcm[g] = out[i]
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
    total_prompts = per_gpu * world
    audio_s = total_prompts * args.steps * SAMPLES_PER_STEP / SAMPLE_RATE
    roof = gemv_roofline(be, runner, max(5, min(40, args.steps // 5)))
    try:
        cp = copy_peak(be)  # streaming-copy rate of this GPU (read + write), beside the spec peak
        roof["measured_copy_peak_gbs"] = cp["kernel"]
        roof["measured_copy_runtime_gbs"] = cp["runtime"]
    except Exception as e:  # noqa: BLE001  (a measurement beside the line, never a reason to lose it)
        roof["measured_copy_peak_gbs"] = None
        print(f"bench: copy peak failed: {e!r}", file=sys.stderr, flush=True)
    graph_nodes = runner.last_graph_nodes()
    dac_nodes = dac.last_graph_nodes() if dac is not None else None
    for xb, rd in dac_workers[R:]:
        rd.close()
        xb.close()
    close_replicas(reps)

    p8 = None  # the 8-prompts-per-GPU line (the 64-prompt batch over 8 GPUs) beside a many-prompt headline
    if args.p8 and per_gpu > 8 and strong:
        barrier_sync(dist, None)
        reps8, pf8, _ = parler_replicas(args, 8, 2, rank, new_backend)
        warm_concurrent(args, reps8)
        barrier_sync(dist, reps8[0][0])
        t80 = time.perf_counter()
        run_replicas(lambda r: (reps8[r][1].generate(args.steps), reps8[r][0].sync()), 2)
        d8 = max_over_ranks(dist, local, time.perf_counter() - t80)
        close_replicas(reps8)
        p8 = {"workload": "Parler-mini Q4_K AR decode, 8 prompts per GPU (2 lock-step replicas x 4)", "ar_ms_per_step": round(1000 * d8 / args.steps, 4),
              "ar_audio_sec_per_s": round(world * 8 * args.steps * SAMPLES_PER_STEP / SAMPLE_RATE / d8, 3)}
    # The legs added in round 5 run guarded on one GPU: a Python-level failure in one of them is reported
    # in its field and does not take the headline line down with it (a device fault still would).  With
    # several ranks a failed leg re-raises: the legs run collectives, and a rank that skipped the rest of
    # a leg's barriers / reductions would pair its next collective with another rank's different one.
    def guarded(name, fn):
        try:
            return fn()
        except Exception as e:  # noqa: BLE001
            if dist is not None:
                raise
            print(f"bench: leg {name} failed: {e!r}", file=sys.stderr, flush=True)
            return {"error": repr(e)}

    # the reference's default sampler (sampler::sample with top_k 50, temperature 1: include/common.h:45-66,
    # src/sampler.cpp:3-69), seeded, on the device (k_sample.hip), at the headline's shape (AR only)
    def leg_sampled():
        barrier_sync(dist, None)
        reps_s, _, _ = parler_replicas(args, per_gpu, R, rank, new_backend)
        try:
            for r, (rb, rr, _) in enumerate(reps_s):
                rr.set_sampling(ttship.sampling(top_k=50, temperature=1.0, seed=0x5EED + rank * R + r))
                rr.generate(2)
            warm_concurrent(args, reps_s)
            barrier_sync(dist, reps_s[0][0])
            ts0 = time.perf_counter()
            run_replicas(lambda r: (reps_s[r][1].generate(args.sampled_steps), reps_s[r][0].sync()), R)
            ds = max_over_ranks(dist, local, time.perf_counter() - ts0)
        finally:
            close_replicas(reps_s)
        sampled = {"workload": f"as the headline's AR decode ({R} replicas x {bl} lock-step prompts per GPU, KV {args.ctx}), with the "
                               "reference's default sampler: seeded top-k 50, temperature 1 (device sampling, k_sample.hip)",
                   "steps": args.sampled_steps, "ar_ms_per_step": round(1000 * ds / args.sampled_steps, 4),
                   "ar_audio_sec_per_s": round(world * per_gpu * args.sampled_steps * SAMPLES_PER_STEP / SAMPLE_RATE / ds, 3)}
        return sampled

    sampled = guarded("parler_sampled_top_k", leg_sampled) if args.sampled_steps > 0 else None
    # the prompt pass the headline leaves out: every prompt's own sentence (perf_battery's 29, prompt g = HARVARD[g % 29])
    # from position 0 -- batched: each replica's prompts as ONE ragged prompt pass (tts_parler_prefill_ragged: every
    # prompt at its own length, tokens equal to its own pass, tests/test_parler_gpu.py), R replicas concurrently; and
    # as TTS.cpp runs it (one prompt per runner pass, R runners concurrently)
    def leg_prompt_pass():
        barrier_sync(dist, None)
        toks_pp = [sentence_tokens(HARVARD[(rank * per_gpu + g) % len(HARVARD)], cfg.prompt_vocab) for g in range(per_gpu)]
        out = {"workload": f"{per_gpu} prompt passes per GPU from position 0, prompt g = perf_battery sentence g % 29 "
                           f"(word-piece-length synthetic ids, {min(map(len, toks_pp))}-{max(map(len, toks_pp))} tokens)"}
        rcfg = ttship.parler_config(batch=bl, max_ctx=256)
        pbes, pruns = [], []
        try:
            pbes += [new_backend() for _ in range(R)]
            pruns += [ttship.Parler(b.iface(), rcfg) for b in pbes]
            for r in range(R):  # warm (code objects, the prefill's GEMM shapes)
                pruns[r].prefill_ragged(toks_pp[r * bl:(r + 1) * bl])
                pbes[r].sync()

            def ppb(r):
                pruns[r].reset()
                pruns[r].prefill_ragged(toks_pp[r * bl:(r + 1) * bl])
                pbes[r].sync()

            barrier_sync(dist, pbes[0])
            tp0 = time.perf_counter()
            run_replicas(ppb, R)
            dtb = max_over_ranks(dist, local, time.perf_counter() - tp0)
        finally:
            for rr in pruns:
                rr.close()
            for b in pbes:
                b.close()
        out.update({"batched": f"{R} replicas x one ragged prompt pass of {bl} prompts (tts_parler_prefill_ragged)",
                    "ms_total": round(1000 * dtb, 3), "end_to_end_audio_sec_per_s_with_prompt_pass": round(audio_s / (dt + dtb), 3)})
        pcfg = ttship.parler_config(batch=1, max_ctx=256)
        pbes, pruns = [], []
        try:
            pbes += [new_backend() for _ in range(R)]
            pruns += [ttship.Parler(b.iface(), pcfg) for b in pbes]
            for rr, b in zip(pruns, pbes):  # warm (code objects)
                rr.prefill(toks_pp[0].reshape(1, -1))
                b.sync()

            def pp(r):
                for g in range(r, per_gpu, R):
                    pruns[r].reset()
                    pruns[r].prefill(toks_pp[g].reshape(1, -1))
                pbes[r].sync()

            barrier_sync(dist, pbes[0])
            tp0 = time.perf_counter()
            run_replicas(pp, R)
            dtp = max_over_ranks(dist, local, time.perf_counter() - tp0)
        finally:
            for rr in pruns:
                rr.close()
            for b in pbes:
                b.close()
        out["one_prompt_per_pass"] = {"workload": f"TTS.cpp's shape: one prompt per runner pass, {R} runners concurrently",
                                      "ms_total": round(1000 * dtp, 3), "ms_per_prompt": round(1000 * dtp * R / per_gpu, 3),
                                      "end_to_end_audio_sec_per_s_with_prompt_pass": round(audio_s / (dt + dtp), 3)}
        return out

    prompt_pass = guarded("prompt_pass", leg_prompt_pass) if args.prompt_pass else None

    # TTS.cpp's generate() shape (parler_tts_runner::generate, src/models/parler/model.cpp:838-858) for the whole
    # prompt set: every prompt's own perf_battery sentence as the prompt pass (one ragged pass per replica,
    # tts_parler_prefill_ragged), the AR decode from there (each prompt at its own position), and the DAC decode --
    # all inside the timed region, on the headline's replicas / DAC workers layout
    def leg_generate_shape():
        barrier_sync(dist, None)
        gcfg = ttship.parler_config(batch=bl, max_ctx=256 + args.steps + 64, arena_bytes=max(4, (bl + 7) // 8 * 4) << 30)
        sents = [sentence_tokens(HARVARD[(rank * per_gpu + g) % len(HARVARD)], gcfg.prompt_vocab) for g in range(per_gpu)]
        gbes, gruns, gdecs = [], [], []
        try:
            for r in range(R):
                gbes.append(new_backend())
                gruns.append(ttship.Parler(gbes[-1].iface(), gcfg))
            while len(gdecs) < W:
                if len(gbes) <= len(gdecs):
                    gbes.append(new_backend())
                gdecs.append(new_dac_for(args, gbes[len(gdecs)], dcfg))
            toks_g = [None] * R
            pcm_g = [None] * per_gpu

            def ar(r):
                gruns[r].reset()
                gruns[r].prefill_ragged(sents[r * bl:(r + 1) * bl])
                toks_g[r] = gruns[r].generate(args.steps)
                gbes[r].sync()

            def dac_w(w):
                xb, rd = gbes[w], gdecs[w]
                for bt in range(w, n_dac_batches, W):
                    gs = list(range(bt * NBD, min(per_gpu, (bt + 1) * NBD)))
                    if len(gs) == 1 or NBD == 1:
                        for g in gs:
                            pcm_g[g] = rd.decode(dac_codes(toks_g[g // bl][g % bl], dcfg.codebook_size))
                    else:
                        out = rd.decode_batch(np.stack([dac_codes(toks_g[g // bl][g % bl], dcfg.codebook_size) for g in gs]))
                        for i, g in enumerate(gs):
                            pcm_g[g] = out[i]
                xb.sync()

            run_replicas(ar, R)  # warm: code objects, step graphs, the prompt pass's shapes
            run_replicas(dac_w, W)
            barrier_sync(dist, gbes[0])
            tg0 = time.perf_counter()
            run_replicas(ar, R)
            tg1 = time.perf_counter()
            run_replicas(dac_w, W)
            barrier_sync(dist, gbes[0])
            tg2 = time.perf_counter()
            dtg = max_over_ranks(dist, local, tg2 - tg0)
            dtg_ar = max_over_ranks(dist, local, tg1 - tg0)
        finally:
            for d_ in gdecs:
                d_.close()
            for rr in gruns:
                rr.close()
            for b in gbes:
                b.close()
        return {"workload": f"TTS.cpp's generate() per prompt, for the whole set: prompt g = perf_battery sentence g % 29 "
                            f"({min(map(len, sents))}-{max(map(len, sents))} word-piece ids) as one ragged prompt pass per replica, "
                            f"then {args.steps} AR steps from each prompt's own position, then DAC-44k, all timed "
                            f"({R} replicas x {bl} prompts, {W} DAC decoders)",
                "audio_sec_per_s": round(audio_s / dtg, 3), "ms_total": round(1000 * dtg, 3),
                "prompt_pass_and_ar_ms": round(1000 * dtg_ar, 3)}

    generate_shape = guarded("parler_generate_shape", leg_generate_shape) if args.prompt_pass and not args.no_dac else None

    def leg_b1():
        # TTS.cpp's serving shape: b1_replicas one-prompt runners with the step coalescer (equal and ragged
        # KV lengths), the same runners each alone, and b1_wide coalesced ragged runners
        b1 = {}
        legs = [("alone", args.b1_replicas, False, False)]
        if args.b1_coalesce:
            legs = [("coalesced", args.b1_replicas, True, False), ("coalesced_ragged", args.b1_replicas, True, True)] + legs
            if args.b1_wide > 0:
                legs.append(("coalesced_ragged_wide", args.b1_wide, True, True))
        for name, n_run, co, rg in legs:
            barrier_sync(dist, None)
            leg = parler_b1_leg(args, rank, local, new_backend, R=n_run, coalesce=co, ragged=rg)
            t = max_over_ranks(dist, local, leg["ms_per_step"])
            leg["ms_per_step"] = t
            leg["ar_audio_sec_per_s"] = round(world * n_run * SAMPLES_PER_STEP / SAMPLE_RATE * 1000.0 / t, 3)
            b1[name] = leg
        return b1

    b1 = guarded("parler_b1", leg_b1) if args.b1_replicas > 0 else None
    kres = None
    if args.kokoro_prompts > 0:
        kb = [new_backend() for _ in range(2)]
        barrier_sync(dist, kb[0])
        kres = kokoro_leg(kb, args, rank, dist, local, world)
        for b in kb:
            b.close()
    ores = None
    if args.orpheus_steps > 0:
        ob = new_backend()
        barrier_sync(dist, ob)
        ores = orpheus_leg(ob, args, rank)
        ob.close()
        # whole-job rate: every rank decoded its own shard; the slowest rank's time sets it
        t = max_over_ranks(dist, local, ores["ms_per_step"])
        ores["ms_per_step"] = t
        ores["tokens_per_s"] = round(world * args.orpheus_batch * 1000.0 / t, 1)
        ores["ar_audio_sec_per_s"] = round(ores["tokens_per_s"] / ORPHEUS_TOK_PER_AUDIO_S, 3)
        ts = max_over_ranks(dist, local, ores["wall_s"])
        ores["audio_sec_per_s"] = round(world * ores["audio_sec_per_gpu"] / ts, 3)
    dres = None
    if args.dia_steps > 0:
        db = new_backend()
        barrier_sync(dist, db)
        dres = dia_leg(db, args)
        db.close()
        t = max_over_ranks(dist, local, dres["ms_per_step"])
        dres["ms_per_step"] = t
        ts = max_over_ranks(dist, local, dres["wall_s"])
        dres["audio_sec_per_s"] = round(world * dres["audio_sec_per_gpu"] / ts, 3)

    dac_roof = None
    if dac is not None:
        # the DAC leg as a whole (all its kernels, W concurrent decoders) against the f64 matrix-core peak:
        # the fused convs carry ~all of its FLOPs (f16 inputs, f64 accumulation on v_mfma_f64_16x16x4f64)
        fl = dac_flops_per_frame(dcfg) * per_gpu * args.steps
        tf = fl / dt_dac / 1e12
        dac_roof = {"bound": "mfma", "achieved": round(tf, 3), "peak": F64_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": round(tf / F64_MFMA_PEAK_TF, 4),
                    "flops_per_frame": dac_flops_per_frame(dcfg), "frames": per_gpu * args.steps,
                    "note": "algorithmic conv FLOPs of the frames decoded (gaps of batched decodes not counted) / DAC wall time per GPU; "
                            "peak = the measured f64 MFMA rate (scripts/mfma_f64_peak.hip)"}
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            # the box's CPU share: OMP_NUM_THREADS is set to it on the GPU box (16 per GPU); else every core we may use
            ncpu = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
            cpu = cpu_baseline(args, ncpu, bl)
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
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "q4_K weights x q8_K activations (int dot, f32 combine); DAC f16 im2col x f32 weights, f64 accumulate",
            "data": "synthetic (deterministic weights in Parler-mini v1 Q4_K and DAC-44k shapes; token ids from Harvard sentences)",
            "config": {"workload": f"Parler-TTS-mini-v1 Q4_K, greedy AR decode + DAC-44k (BASELINE configs[2]) over the fixed "
                                   f"{total_prompts}-prompt set", "model": "parler-tts-mini-v1", "prompts_per_gpu": per_gpu,
                       "global_batch": total_prompts, "kv_len_start": args.ctx, "frames_per_prompt": args.steps,
                       "parallelism": f"dp{world} (prompt shards), {R} concurrent replicas x {bl} lock-step prompts per GPU, "
                                      f"{W} concurrent DAC decoders" + (f" of {NBD} prompts per batched decode" if NBD > 1 else ""),
                       "graph_nodes_per_step": graph_nodes, "dac_graph_nodes": dac_nodes},
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
            "parler_8_prompts_per_gpu": p8,
            "parler_sampled_top_k": sampled,
            "prompt_pass": prompt_pass,
            "parler_generate_shape": generate_shape,
            "parler_b1": b1,
            "kokoro": kres,
            "orpheus": ores,
            "dia": dres,
            "roofline": roof,
            "roofline_dac": dac_roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
