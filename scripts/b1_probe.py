"""The bench's coalesced B = 1 leg alone (R one-prompt runners on their own threads, TTS.cpp's step loop),
for a kernel trace of the executor's batched steps.  Usage: b1_probe.py [R] [steps] [ragged 0/1]"""
import argparse
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "tts.cpp_amd"))
import ttship  # noqa: E402
import bench  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ragged = len(sys.argv) > 3 and sys.argv[3] == "1"
    args = argparse.Namespace(b1_replicas=R, b1_steps=steps, ctx=448, warmup=5)
    out = bench.parler_b1_leg(args, 0, 0, lambda: ttship.HipBackend(0), R=R, coalesce=True, ragged=ragged)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
