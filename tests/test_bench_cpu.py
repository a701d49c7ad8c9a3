"""bench.py's host-side rules (no device): prompts per batched DAC decode."""
import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def ns(**kw):
    base = dict(dac_batch=None, steps=20, per_gpu_=64)
    base.update(kw)
    return argparse.Namespace(**base)


def test_dac_batch_rule():
    assert bench.dac_batch(ns()) == 8            # 64 prompts per GPU, short sequences: 8 per decode
    assert bench.dac_batch(ns(per_gpu_=32)) == 8
    assert bench.dac_batch(ns(per_gpu_=8)) == 4  # the 8-GPU share: two decoders of 4
    assert bench.dac_batch(ns(per_gpu_=2)) == 1
    assert bench.dac_batch(ns(steps=861)) == 1   # long sequences one by one
    assert bench.dac_batch(ns(steps=64)) == 8 and bench.dac_batch(ns(steps=65)) == 1
    assert bench.dac_batch(ns(dac_batch=3, steps=861)) == 3  # an explicit --dac-batch wins
    assert bench.dac_batch(ns(dac_batch=0)) == 1
