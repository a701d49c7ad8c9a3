"""Kokoro-82M end to end (tokens -> durations -> PCM) on one GPU, synthetic weights in the real shapes.

One JSON line per prompt length: ms for the duration graph, the main graph (decoder + generator)
and the whole run (both graphs + the host mask step + PCM readback), audio-seconds per wall-second.
Usage: python scripts/bench_kokoro_model.py [n_tokens ...]   (default 16 64)
"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
import ttship  # noqa: E402


def timed(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    return (time.perf_counter() - t0) / reps, out


def main():
    lens = [int(a) for a in sys.argv[1:]] or [16, 64]
    be = ttship.HipBackend(0)
    cfg = ttship.kokoro_config(max_tokens=max(max(lens), 16), max_total=max(lens) * 12)
    k = ttship.Kokoro(be.iface(), cfg)
    rng = np.random.default_rng(0)
    for n in lens:
        toks = rng.integers(1, cfg.n_vocab, n).astype(np.int32)
        toks[0] = toks[-1] = 0
        dt_d, (hidden, lengths) = timed(lambda: k.durations(toks), 5)
        dt_m, pcm = timed(lambda: k.decode(toks, hidden, lengths), 3)
        dt_r, pcm2 = timed(lambda: k.run(toks), 3)
        audio = pcm2.shape[0] / cfg.gen.sample_rate
        print(json.dumps({"model": "kokoro-82m", "tokens": n, "frames": int(lengths.sum()), "audio_s": round(audio, 3),
                          "ms_durations": round(1000 * dt_d, 3), "ms_decode": round(1000 * dt_m, 3), "ms_run": round(1000 * dt_r, 3),
                          "audio_sec_per_s": round(audio / dt_r, 2), "nodes": [k.last_graph_nodes(0), k.last_graph_nodes(1)],
                          "pcm_std": round(float(np.std(pcm2)), 4)}), flush=True)
    k.close()
    be.close()


if __name__ == "__main__":
    main()
