"""Multi-rank path of bench.py on CPU: world_size 2 over gloo, each rank stepping its prompt shard
through the oracle backend (the same C++ Parler runner the GPU uses).  Checks that the shards are the
matching rows of the whole batch, that the max-over-ranks timing reduction works, that the token
gather to rank 0 reproduces a single-process run of the whole batch exactly, and that the final audio
gather (ragged per-prompt PCM, all-gathered lengths + point-to-point gatherv) arrives in prompt order."""
import os
import pathlib
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

CFG = dict(n_layers=2, hidden=256, heads=4, ffn=1024, max_ctx=64, prompt_vocab=512, max_positions=80)
PER_RANK, PROMPT_LEN, STEPS = 2, 6, 4


def _run(batch, offset, n_threads=2):
    import bench
    import py_oracle
    import ttship
    cfg = ttship.parler_config(batch=batch, **CFG)
    p = ttship.Parler(py_oracle.iface(n_threads), cfg)
    try:
        p.prefill(bench.prompt_tokens(batch, PROMPT_LEN, cfg.prompt_vocab, offset=offset))
        return p.generate(STEPS)
    finally:
        p.close()


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for p in (ROOT, ROOT / "tts.cpp_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    import bench
    r, w, local, dist = bench.dist_init(backend="gloo")
    try:
        toks = _run(PER_RANK, offset=r * PER_RANK)
        bench.barrier_sync(dist, None)
        dt = bench.max_over_ranks(dist, local, 1.0 + r)
        full = bench.gather_tokens(dist, r, w, local, toks)
        # audio gather: ragged per-prompt PCM lengths, rank-tagged values
        pcms = [np.full(100 + 37 * i + 11 * r, r * 10 + i, dtype=np.float32) for i in range(PER_RANK)]
        audio = bench.gather_audio(dist, r, w, local, pcms)
        q.put((r, dt, full, audio))
    finally:
        dist.destroy_process_group()


def test_prompt_shards_are_rows_of_the_batch():
    import bench
    whole = bench.prompt_tokens(2 * PER_RANK, PROMPT_LEN, 512)
    assert np.array_equal(bench.prompt_tokens(PER_RANK, PROMPT_LEN, 512, offset=PER_RANK), whole[PER_RANK:])


def test_two_rank_gloo_gather_matches_single_process():
    world, port = 2, 29611
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, dt, full, audio = q.get(timeout=300)
        got[r] = (dt, full, audio)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(dt == pytest.approx(2.0) for dt, _, _ in got.values())   # max over ranks
    assert got[1][1] is None and got[1][2] is None
    audio = got[0][2]  # global prompt order, each prompt's own length and values
    assert len(audio) == world * PER_RANK
    for g, a in enumerate(audio):
        r, i = divmod(g, PER_RANK)
        assert a.shape == (100 + 37 * i + 11 * r,) and np.all(a == r * 10 + i)
    ref = _run(world * PER_RANK, offset=0)
    assert got[0][1].shape == ref.shape
    assert np.array_equal(got[0][1], ref)
