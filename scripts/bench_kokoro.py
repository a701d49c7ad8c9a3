"""Kokoro-82M iSTFTNet generator throughput on one GPU (synthetic weights in the real shapes).

One JSON line per frame count: ms per generator call (host uv/noise/envelope prep + upload +
graph + PCM readback) and audio-seconds per wall-second (300 samples @ 24 kHz per input frame).
Usage: python scripts/bench_kokoro.py [frames ...]   (default 80 800 = 1 s and 10 s of audio)
"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402


def main():
    frames = [int(a) for a in sys.argv[1:]] or [80, 800]
    be = ttship.HipBackend(0)
    cfg = ttship.kokoro_gen_config(max_frames=max(frames))
    k = ttship.KokoroGenerator(be.iface(), cfg)
    rng = np.random.default_rng(0)
    for T in frames:
        x = (rng.standard_normal((T, cfg.in_channels)) * 0.5).astype(np.float32)
        f0 = rng.uniform(80, 250, T).astype(np.float32)
        style = rng.standard_normal(cfg.style_dim).astype(np.float32)
        rand = rng.random((cfg.harmonic_num + 1, 300 * T), dtype=np.float32)
        pcm = np.empty(300 * T, dtype=np.float32)
        k.run(x, f0, style, rand, out=pcm)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            k.run(x, f0, style, rand, out=pcm)
        dt = (time.perf_counter() - t0) / reps
        audio = T * 300 / cfg.sample_rate
        print(json.dumps({"model": "kokoro-82m-generator", "frames": T, "audio_s": audio, "ms_per_call": round(1000 * dt, 3),
                          "audio_sec_per_s": round(audio / dt, 2), "nodes": k.last_graph_nodes(),
                          "pcm_std": round(float(np.std(pcm)), 4)}), flush=True)
    k.close()
    be.close()


if __name__ == "__main__":
    main()
