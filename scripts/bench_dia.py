"""Dia-1.6B Q8_0 decode throughput on one GPU (BASELINE configs[3]): synthetic weights in the exact
shapes, the encoder step over a Harvard-sentence prompt, then timed CFG decoder steps (greedy heads
fed back).  Dia produces one 9-codebook DAC frame (512 samples at 44.1 kHz) per step.
usage: bench_dia.py [steps] [decoder_layers]"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    kw = {"n_decoder_layers": int(sys.argv[2])} if len(sys.argv) > 2 else {}
    be = ttship.HipBackend(0)
    d = ttship.Dia(be.iface(), ttship.dia_config(**kw))
    text = np.frombuffer(b"\x01 The birch canoe slid on the smooth planks. Glue the sheet to the dark blue background.",
                         dtype=np.uint8).astype(np.int32)
    t0 = time.perf_counter()
    lg = d.prefill(text, np.full(9, 1026, dtype=np.int32))
    t_enc = time.perf_counter() - t0
    audio = lg.argmax(axis=1).astype(np.int32)
    for _ in range(3):
        audio = d.decode(audio).argmax(axis=1).astype(np.int32)
    t0 = time.perf_counter()
    for _ in range(steps):
        audio = d.decode(audio).argmax(axis=1).astype(np.int32)
    dt = time.perf_counter() - t0
    be.set_option(ttship.OPT["PROFILE_GEMV"], 1)
    be.gemv_stats(-1, reset=True)
    for _ in range(4):
        audio = d.decode(audio).argmax(axis=1).astype(np.int32)
    ms, n, nbytes = be.gemv_stats(ttship.Q8_0, reset=True)
    be.set_option(ttship.OPT["PROFILE_GEMV"], 0)
    us = 1000 * ms / max(n, 1)
    print(json.dumps({"workload": "Dia-1.6B Q8_0 CFG decode (BASELINE configs[3]), synthetic weights",
                      "ms_per_step": round(1000 * dt / steps, 3), "audio_sec_per_s": round(steps * 512 / 44100 / dt, 3),
                      "encoder_step_ms": round(1000 * t_enc, 1), "weight_GB": round(d.weight_bytes() / 1e9, 3),
                      "q8_0_gemv": {"avg_launch_us": round(us, 2), "GBps": round(nbytes / max(n, 1) / (us * 1e-6) / 1e9, 1),
                                    "launches": n}}), flush=True)
    d.close()
    be.close()


if __name__ == "__main__":
    main()
