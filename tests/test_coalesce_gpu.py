"""The step coalescer (tts.cpp_amd/csrc/coalesce.hip) on TTS.cpp's own serving shape.

TTS.cpp's server runs one runner per worker thread, each with its own backend and model copy
(/root/reference/examples/server/server.cpp:316-321,885-895), and a runner decodes one sequence per
step graph (parler_tts_runner::decode, /root/reference/src/models/parler/model.cpp:648-693): the
runners here are driven exactly so -- one backend and one runner per host thread, TTS.cpp's step
loop (graph_compute, logits read back at once, host sampler) -- and the backend coalesces their
decode steps into batched launches.  Every runner's tokens must equal the same runner decoding
alone and the CPU oracle's (bit-exact), with coalesced launches actually taken."""
import threading
import time

import numpy as np
import pytest

import py_oracle
import ttship


@pytest.fixture(autouse=True)
def coalescer_on():
    """The coalescer is on by default (tts_hip_coalesce_enable); kept on for these tests whatever the
    environment says, then back to what it was."""
    prev = ttship.coalesce_enable(True)
    yield
    ttship.coalesce_enable(prev)


TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=128, prompt_vocab=512,
            max_positions=160)


def run_threads(fn, n):
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


def prompt(r, n=7, vocab=512):
    return ((np.arange(n, dtype=np.int32) * (31 + 2 * r) + 5 * r + 1) % vocab).reshape(1, n)


def serve(ifaces, cfg, prompts, steps, stagger_s=0.0, cfgs=None):
    """One runner per iface, prefilled with its prompt, then `steps` decode steps from one thread per
    runner (the server's workers; runner i starts i * stagger_s seconds after runner 0); returns every
    runner's tokens."""
    runs = [ttship.Parler(it, (cfgs[i] if cfgs else cfg)) for i, it in enumerate(ifaces)]
    try:
        for r, p in zip(runs, prompts):
            r.prefill(p)
        out = [None] * len(runs)

        def go(i):
            if stagger_s:
                time.sleep(i * stagger_s)
            out[i] = runs[i].generate(steps)

        run_threads(go, len(runs))
        return out
    finally:
        for r in runs:
            r.close()


def oracle_tokens(cfg, p, steps):
    c = ttship.Parler(py_oracle.iface(8), cfg)
    try:
        c.prefill(p)
        return c.generate(steps)
    finally:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 5])
def test_coalesced_runners_match_alone_and_oracle(n):
    cfg = ttship.parler_config(batch=1, **TINY)
    prompts = [prompt(r) for r in range(n)]
    bes = [ttship.HipBackend(0) for _ in range(n)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([b.iface(reference_flow=True) for b in bes], cfg, prompts, 12)
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    carried = after["member_steps"] - before["member_steps"]
    assert carried >= n * 6, f"{before} {after}"  # most steps ran coalesced
    # each runner alone (coalescing off) and on the oracle
    for r in range(n):
        be = ttship.HipBackend(0)
        be.set_option(ttship.OPT["COALESCE"], 0)
        try:
            alone = serve([be.iface(reference_flow=True)], cfg, [prompts[r]], 12)[0]
        finally:
            be.close()
        c = ttship.Parler(py_oracle.iface(8), cfg)
        try:
            c.prefill(prompts[r])
            ref = c.generate(12)
        finally:
            c.close()
        assert np.array_equal(got[r], alone), f"runner {r}: coalesced vs alone\n{got[r]}\n{alone}"
        assert np.array_equal(got[r], ref), f"runner {r}: coalesced vs oracle\n{got[r]}\n{ref}"


@pytest.mark.gpu
def test_runners_at_different_lengths_coalesce_exact():
    """Runners whose KV lengths differ share launches (each attention at its own key count, each KV
    store at its own position), and every runner's tokens stay the oracle's."""
    cfg = ttship.parler_config(batch=1, **TINY)
    prompts = [prompt(0, 7), prompt(1, 7), prompt(2, 9)]
    bes = [ttship.HipBackend(0) for _ in range(3)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([b.iface(reference_flow=True) for b in bes], cfg, prompts, 8)
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    assert after["ragged_launches"] > before["ragged_launches"], f"{before} {after}"
    assert after["member_steps"] - before["member_steps"] >= 3 * 4, f"{before} {after}"
    for r in range(3):
        assert np.array_equal(got[r], oracle_tokens(cfg, prompts[r], 8)), f"runner {r}"


@pytest.mark.gpu
def test_staggered_runners_at_four_lengths():
    """TTS.cpp's server shape: 4 workers, 4 prompts of different lengths, decoding from 4 threads that
    start at different times.  Most steps run coalesced (at 4 different KV lengths), and every runner's
    tokens are its own oracle B = 1 run's."""
    cfg = ttship.parler_config(batch=1, **TINY)
    steps = 24
    prompts = [prompt(r, 5 + 4 * r) for r in range(4)]
    bes = [ttship.HipBackend(0) for _ in range(4)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([b.iface(reference_flow=True) for b in bes], cfg, prompts, steps, stagger_s=0.01)
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    carried = after["member_steps"] - before["member_steps"]
    assert carried >= 4 * steps // 2, f"{before} {after}"  # most steps coalesced
    assert after["ragged_launches"] > before["ragged_launches"], f"{before} {after}"
    for r in range(4):
        assert np.array_equal(got[r], oracle_tokens(cfg, prompts[r], steps)), f"runner {r}"


@pytest.mark.gpu
def test_two_kinds_of_graphs_coalesce_separately():
    """Two model configurations (2 and 3 layers) served at once, two runners each, at different prompt
    lengths: each kind of step graph coalesces with its own kind (several groups per rendezvous), and
    every runner's tokens are the oracle's."""
    cfg2 = ttship.parler_config(batch=1, **TINY)
    cfg3 = ttship.parler_config(batch=1, **dict(TINY, n_layers=3))
    cfgs = [cfg2, cfg3, cfg2, cfg3]
    prompts = [prompt(r, 6 + r) for r in range(4)]
    bes = [ttship.HipBackend(0) for _ in range(4)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([b.iface(reference_flow=True) for b in bes], None, prompts, 10, cfgs=cfgs)
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    assert after["member_steps"] - before["member_steps"] >= 4 * 5, f"{before} {after}"
    for r in range(4):
        assert np.array_equal(got[r], oracle_tokens(cfgs[r], prompts[r], 10)), f"runner {r}"


@pytest.mark.gpu
def test_generic_head_dim_coalesced():
    """A head dim the row / split attention kernels do not take (32): the generic decode attention
    kernel runs the coalesced step, with its private copy of each member's output in place."""
    cfg = ttship.parler_config(batch=1, **dict(TINY, n_attn_heads=8))
    prompts = [prompt(r, 6 + 2 * r) for r in range(3)]
    bes = [ttship.HipBackend(0) for _ in range(3)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([b.iface(reference_flow=True) for b in bes], cfg, prompts, 8)
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    assert after["member_steps"] - before["member_steps"] >= 3 * 4, f"{before} {after}"
    for r in range(3):
        assert np.array_equal(got[r], oracle_tokens(cfg, prompts[r], 8)), f"runner {r}"


@pytest.mark.gpu
def test_weights_that_differ_are_not_shared():
    """Two runners with different weights (another seed) submit the same step graph: the content check
    refuses to read one copy for both, so each runs its own step and keeps its own tokens."""
    cfg_a = ttship.parler_config(batch=1, **TINY)
    cfg_b = ttship.parler_config(batch=1, seed=0x5EED + 77, **TINY)
    bes = [ttship.HipBackend(0) for _ in range(2)]
    try:
        before = ttship.coalesce_stats(0)
        runs = [ttship.Parler(bes[0].iface(reference_flow=True), cfg_a), ttship.Parler(bes[1].iface(reference_flow=True), cfg_b)]
        try:
            for r in runs:
                r.prefill(prompt(0))
            out = [None, None]

            def go(i):
                out[i] = runs[i].generate(6)

            run_threads(go, 2)
        finally:
            for r in runs:
                r.close()
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    assert after["launches"] == before["launches"], f"{before} {after}"
    for cfg, tok in ((cfg_a, out[0]), (cfg_b, out[1])):
        c = ttship.Parler(py_oracle.iface(8), cfg)
        try:
            c.prefill(prompt(0))
            assert np.array_equal(tok, c.generate(6))
        finally:
            c.close()


@pytest.mark.gpu
def test_parler_mini_8_runners_coalesced_bit_identical():
    """Parler-mini Q4_K (full shapes), 8 one-prompt runners at 8 different prompt lengths on 8 backends
    from 8 threads: tokens bit-identical to each runner decoding alone."""
    cfg = ttship.parler_config(batch=1, max_ctx=256)
    n, steps = 8, 10
    prompts = [prompt(r, 12 + r, cfg.prompt_vocab) for r in range(n)]
    bes = [ttship.HipBackend(0) for _ in range(n)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([b.iface(reference_flow=True) for b in bes], cfg, prompts, steps)
        after = ttship.coalesce_stats(0)
    finally:
        for b in bes:
            b.close()
    assert after["member_steps"] - before["member_steps"] >= n * (steps // 2), f"{before} {after}"
    assert after["max_group"] >= 4, after
    assert after["ragged_launches"] > before["ragged_launches"], f"{before} {after}"
    be = ttship.HipBackend(0)
    be.set_option(ttship.OPT["COALESCE"], 0)
    try:
        for r in (0, 3, 7):
            alone = serve([be.iface(reference_flow=True)], cfg, [prompts[r]], steps)[0]
            assert np.array_equal(got[r], alone), f"runner {r}"
    finally:
        be.close()


@pytest.mark.gpu
def test_adapter_runners_from_threads_coalesce_and_match_oracle():
    """TTS.cpp's own path: one ggml backend per server worker (the adapter, reached through the ggml
    registry and vtables, tests/ggml_stub/adapter_harness.cpp), one one-prompt Parler runner on each,
    decoding from its own thread with logits read back every step and the host sampler.  Their step
    graphs coalesce inside the adapter's graph_compute, and every runner's tokens are the CPU oracle's
    at batch 1."""
    from test_adapter_gpu import AdapterBackend
    n, steps = 4, 12
    cfg = ttship.parler_config(batch=1, **TINY)
    prompts = [prompt(r) for r in range(n)]
    ads = [AdapterBackend(0) for _ in range(n)]
    try:
        before = ttship.coalesce_stats(0)
        got = serve([a.iface() for a in ads], cfg, prompts, steps)
        after = ttship.coalesce_stats(0)
        for a in ads:
            s = a.stats()
            assert s["compute_failures"] == 0 and s["refused"] == 0, (s, a.last_refused())
    finally:
        for a in ads:
            a.close()
    assert after["member_steps"] - before["member_steps"] >= n * (steps // 2), f"{before} {after}"
    for r in range(n):
        c = ttship.Parler(py_oracle.iface(8), cfg)
        try:
            c.prefill(prompts[r])
            assert np.array_equal(got[r], c.generate(steps)), f"runner {r}"
        finally:
            c.close()
