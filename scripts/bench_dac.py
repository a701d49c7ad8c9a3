"""DAC-44k decoder throughput on one GPU (synthetic weights in the real shapes).

Prints one JSON line per (frames, accumulation mode): ms per decode and audio-seconds per
wall-second (512 samples @ 44.1 kHz per latent frame).
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
    frames = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [50, 861]
    modes = ((0, 1),) if "--default-only" in sys.argv else ((0, 1), (0, 0), (1, 1))
    be = ttship.HipBackend(0)
    cfg = ttship.dac_config(max_frames=max(frames))
    dac = ttship.Dac(be.iface(), cfg)
    rng = np.random.default_rng(0)
    for f32acc, convt in modes:
        be.set_option(3, f32acc)
        be.set_option(4, convt)
        for T in frames:
            codes = rng.integers(0, cfg.codebook_size, size=(T, cfg.n_codebooks))
            dac.decode(codes)
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                pcm = dac.decode(codes)
            dt = (time.perf_counter() - t0) / reps
            audio = T * dac.hop / 44100.0
            print(json.dumps({"frames": T, "conv_f32acc": f32acc, "convt_lds": convt, "ms_per_decode": round(1000 * dt, 3),
                              "audio_sec_per_s": round(audio / dt, 2), "nodes": dac.last_graph_nodes(),
                              "pcm_std": round(float(np.std(pcm)), 4)}), flush=True)
    be.set_option(3, 0)
    be.set_option(4, 1)
    dac.close()
    be.close()


if __name__ == "__main__":
    main()
