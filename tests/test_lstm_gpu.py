"""Kokoro LSTM on the HIP backend vs the CPU oracle.

The graph is the reference's unrolled recurrence (tests/lstm.py = build_lstm_run node for node).
With TTS_FUSE_LSTM the planner turns each chain into one k_lstm_step launch per time step plus one
output write; the per-step arithmetic keeps ggml's rounding sequence (f64 dot accumulation, every
add / activation rounded to f32), so the outputs match the oracle to the f64-reassociation level:
identical in almost every element, <= 2e-6 anywhere (the recurrence can carry a 1-ulp difference
forward).  The unfused generic path is checked the same way.
"""
import numpy as np
import pytest

import lstm
import nodes as nd
import ttship

F32, F16 = ttship.F32, ttship.F16


def run_both(hip, build):
    g1, g2 = nd.Graph(), nd.Graph()
    o1, o2 = build(g1), build(g2)
    g1.run_hip(hip)
    g2.run_oracle(n_threads=8)
    return g1.node_array(o1), g2.node_array(o2)


def check(gpu, ref, tol=2e-6):
    err = float(np.max(np.abs(gpu.astype(np.float64) - ref.astype(np.float64))))
    frac = float(np.mean(gpu != ref))
    assert err <= tol and frac <= 0.01, f"max err {err:.3e}, mismatching fraction {frac:.3e}"


CASES = [  # T, n_in, hidden, bidirectional, weight type
    (37, 640, 256, True, F32),     # Kokoro predictor LSTM shape
    (128, 512, 256, True, F32),    # Kokoro text-encoder LSTM shape
    (20, 640, 256, True, F16),
    (1, 64, 32, True, F32),        # a single step: no concat chain
    (9, 24, 16, False, F32),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_lstm_fused(hip, case):
    T, n_in, hd, bi, wt = case
    rng = np.random.default_rng(T)
    x = (rng.standard_normal((T, n_in)) * 0.5).astype(np.float32)
    dirs = lstm.lstm_weights(T + 1, n_in, hd, bidirectional=bi)
    before = hip.counters()
    gpu, ref = run_both(hip, lambda g: lstm.lstm(g, x, dirs, wtype=wt))
    after = hip.counters()
    n_dir = 2 if bi else 1
    assert after["lstm_chains"] - before["lstm_chains"] == n_dir
    assert after["lstm_steps"] - before["lstm_steps"] == n_dir * T
    check(gpu, ref)
    # and the graph means nn.LSTM
    want = lstm.ref_lstm(x if wt == F32 else x, dirs)
    assert np.max(np.abs(ref.reshape(T, -1) - want)) < (2e-5 if wt == F32 else 3e-3)


@pytest.mark.gpu
def test_lstm_unfused_generic_path(hip):
    T, n_in, hd = 12, 64, 32
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((T, n_in)) * 0.5).astype(np.float32)
    dirs = lstm.lstm_weights(6, n_in, hd)
    hip.set_option(0, ttship.FUSE_ALL & ~64)
    try:
        before = hip.counters()
        gpu, ref = run_both(hip, lambda g: lstm.lstm(g, x, dirs))
        assert hip.counters()["lstm_steps"] == before["lstm_steps"]
    finally:
        hip.set_option(0, ttship.FUSE_ALL)
    check(gpu, ref)


@pytest.mark.gpu
def test_lstm_not_fused_when_intermediate_escapes(hip):
    """An intermediate read outside the chain (here a partial concat) keeps the generic path."""
    T, n_in, hd = 6, 32, 16
    rng = np.random.default_rng(9)
    x = (rng.standard_normal((T, n_in)) * 0.5).astype(np.float32)
    dirs = lstm.lstm_weights(10, n_in, hd, bidirectional=False)

    def build(g):
        xl = g.leaf(x)
        z = g.leaf(np.zeros(hd, np.float32))
        out, h, c = lstm.lstm_run(g, xl, z, z, dirs[0])
        side = g.node("SCALE", F32, [hd, 1], [c], fparams={0: 2.0})  # c_last read outside the chain
        return g.node("CONCAT", F32, [hd, T + 1], [out, side], params=[1])
    before = hip.counters()
    gpu, ref = run_both(hip, build)
    assert hip.counters()["lstm_steps"] == before["lstm_steps"]
    check(gpu, ref)
