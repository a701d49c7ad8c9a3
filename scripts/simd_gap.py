"""Scalar-vs-SIMD oracle gap (host only, no device).  The oracle (and so the GPU, which matches it
bit for bit) follows ggml-cpu's generic scalar loops; a stock x86 ggml-cpu build runs the AVX2 / FMA /
F16C variants instead (oracle_set_simd_mode(1), oracle/ggml_ref.c).  This runs the same graphs in
both modes and prints one JSON line per workload:
  dac      DAC-44k decoder at full shapes, T latent frames: max / rms |PCM_scalar - PCM_simd|
  kokoro   Kokoro-82M end to end (F32 and F16 weights), one prompt, the main graph run from the
           scalar durations in both modes (rounded lengths compared separately): PCM deltas
  kokoro_gen  the Kokoro-82M iSTFTNet generator alone on fixed inputs (no duration / F0 path): the
           conv stack's own delta
  parler   Parler-mini Q4_K greedy decode, batch 1: the first step whose tokens differ
  dia      Dia-1.6B shapes (2 layers, Q8_0) greedy decode: the first step whose argmax differs
With --gpu (on the GPU box) the DAC and the Kokoro generator also run on the HIP backend with the
f64 conv accumulation (default) and with TTS_HIP_OPT_CONV_F32ACC = 2, each compared with both oracle
modes.
Usage: python3 scripts/simd_gap.py [dac_frames] [parler_steps] [threads] [--gpu]"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for d in ("tts.cpp_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / d))
import py_oracle  # noqa: E402
import ttship  # noqa: E402


def both(fn):
    with py_oracle.simd_mode(0):
        a = fn()
    with py_oracle.simd_mode(1):
        b = fn()
    return a, b


def pcm_gap(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return {"max_abs": float(d.max()), "rms": float(np.sqrt(np.mean(d * d))), "peak": float(np.max(np.abs(a))),
            "frac_over_1e-4": float(np.mean(d > 1e-4))}


def dac(T, nt):
    cfg = ttship.dac_config(max_frames=T)
    codes = np.random.default_rng(11).integers(0, cfg.codebook_size, size=(T, cfg.n_codebooks))
    d = ttship.Dac(py_oracle.iface(nt), cfg)
    try:
        t0 = time.time()
        a, b = both(lambda: d.decode(codes))
        return dict(workload="dac-44k", frames=T, seconds=round(time.time() - t0, 1), **pcm_gap(a, b))
    finally:
        d.close()


def kokoro(wtype, n, nt):
    from test_kokoro_model_cpu import tokens
    cfg = ttship.kokoro_config(max_tokens=48, max_total=256, weight_type=wtype)
    toks = tokens(n, 5)
    k = ttship.Kokoro(py_oracle.iface(nt), cfg)
    try:
        t0 = time.time()
        (h0, l0), (h1, l1) = both(lambda: k.durations(toks))
        rand = np.random.default_rng(12).random((cfg.gen.harmonic_num + 1, 600 * int(l0.sum())), dtype=np.float32)
        a, b = both(lambda: k.decode(toks, h0, l0, rand))
        return dict(workload="kokoro-82m", weights="f16" if wtype == ttship.F16 else "f32", tokens=n,
                    lengths_equal=bool(np.array_equal(l0, l1)), hidden_max_abs=float(np.max(np.abs(h0 - h1))),
                    seconds=round(time.time() - t0, 1), **pcm_gap(a, b))
    finally:
        k.close()


def kokoro_gen(T, nt):
    from test_kokoro_cpu import inputs
    cfg = ttship.kokoro_gen_config(max_frames=T)
    args = inputs(cfg, T, 3)

    def run():
        k = ttship.KokoroGenerator(py_oracle.iface(nt), cfg)
        try:
            return k.run(*args)
        finally:
            k.close()
    t0 = time.time()
    a, b = both(run)
    return dict(workload="kokoro-82m-generator", frames=T, seconds=round(time.time() - t0, 1), **pcm_gap(a, b))


def gpu_legs(T, nt):
    """HIP f64 / f32-batch conv accumulation vs the scalar and SIMD oracles (DAC-44k, Kokoro generator)."""
    from test_kokoro_cpu import inputs
    hip = ttship.HipBackend(0)
    out = []
    try:
        dcfg = ttship.dac_config(max_frames=T)
        codes = np.random.default_rng(11).integers(0, dcfg.codebook_size, size=(T, dcfg.n_codebooks))
        kcfg = ttship.kokoro_gen_config(max_frames=4)
        kargs = inputs(kcfg, 4, 3)

        def dac_on(iface):
            d = ttship.Dac(iface, dcfg)
            try:
                return d.decode(codes)
            finally:
                d.close()

        def gen_on(iface):
            k = ttship.KokoroGenerator(iface, kcfg)
            try:
                return k.run(*kargs)
            finally:
                k.close()
        for name, fn in (("dac-44k", dac_on), ("kokoro-82m-generator", gen_on)):
            ref0, ref1 = both(lambda: fn(py_oracle.iface(nt)))
            for acc in (0, 2):
                hip.set_option(ttship.OPT["CONV_F32ACC"], acc)
                g = fn(hip.iface())
                hip.set_option(ttship.OPT["CONV_F32ACC"], 0)
                out.append({"workload": name, "gpu_conv": "f64" if acc == 0 else "f32-per-32-batch",
                            "vs_scalar_oracle": pcm_gap(ref0, g)["max_abs"], "vs_simd_oracle": pcm_gap(ref1, g)["max_abs"],
                            "scalar_vs_simd": pcm_gap(ref0, ref1)["max_abs"]})
    finally:
        hip.close()
    return out


def parler(steps, nt):
    cfg = ttship.parler_config(max_ctx=steps + 64, batch=1)
    prompt = (np.arange(24, dtype=np.int32).reshape(1, 24) * 131) % cfg.prompt_vocab

    def run():
        p = ttship.Parler(py_oracle.iface(nt), cfg)
        try:
            p.set_device_sampling(False)
            p.prefill(prompt)
            return p.generate(steps)[0]
        finally:
            p.close()
    t0 = time.time()
    a, b = both(run)
    diff = np.nonzero(np.any(a != b, axis=1))[0]
    return {"workload": "parler-mini-q4_k", "steps": steps, "seconds": round(time.time() - t0, 1),
            "first_divergent_step": int(diff[0]) if diff.size else None, "steps_differing": int(diff.size)}


def dia(steps, nt):
    cfg = ttship.dia_config(n_decoder_layers=2, n_encoder_layers=1)
    text = np.frombuffer(b"[S1] Hello there. [S2] Hi, how are you doing today?", dtype=np.uint8).astype(np.int32)

    def run():
        d = ttship.Dia(py_oracle.iface(nt), cfg)
        try:
            d.prefill(text, np.full(cfg.n_output_heads, 1026, dtype=np.int32))
            return d.generate(np.full(cfg.n_output_heads, 1026, dtype=np.int32), steps)
        finally:
            d.close()
    t0 = time.time()
    a, b = both(run)
    diff = np.nonzero(np.any(a != b, axis=1))[0]
    return {"workload": "dia-1.6b-widths-2-decoder-layers-q8_0", "steps": steps, "seconds": round(time.time() - t0, 1),
            "first_divergent_step": int(diff[0]) if diff.size else None, "steps_differing": int(diff.size)}


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    T = int(argv[0]) if len(argv) > 0 else 6
    steps = int(argv[1]) if len(argv) > 1 else 40
    nt = int(argv[2]) if len(argv) > 2 else 8
    if "--gpu" in sys.argv:
        for r in gpu_legs(T, nt):
            print(json.dumps(r), flush=True)
        return
    for job in (lambda: dac(T, nt), lambda: kokoro_gen(4, nt), lambda: kokoro(ttship.F32, 12, nt),
                lambda: kokoro(ttship.F16, 12, nt), lambda: parler(steps, nt), lambda: dia(16, nt)):
        print(json.dumps(job()), flush=True)


if __name__ == "__main__":
    main()
