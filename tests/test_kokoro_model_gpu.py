"""Kokoro end to end on the HIP backend vs the CPU oracle on the same graphs and synthetic weights.

Bars (north_star): the duration graph's rounded lengths identical (they size everything after
them), PCM within 1e-4 absolute.  The main graph runs from the oracle's durations on both sides so
the PCM comparison isolates it; run() is then checked to chain the two graphs exactly as
durations() + decode() do.  The oracle itself is checked against a PyTorch restatement of Kokoro in
tests/test_kokoro_model_cpu.py."""
import numpy as np
import pytest

import py_oracle
import ttship
from test_kokoro_model_cpu import TINY, tokens

CFGS = {
    "tiny": dict(TINY),
    "kokoro82m": dict(max_tokens=16, max_total=64),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,seed,wtype", [("tiny", 7, 0, ttship.F32), ("tiny", 13, 1, ttship.F32), ("kokoro82m", 6, 2, ttship.F32),
                                               ("tiny", 11, 3, ttship.F16), ("kokoro82m", 6, 2, ttship.F16),
                                               ("kokoro82m", 40, 5, ttship.F16)])
def test_kokoro_model_matches_oracle(hip, name, n, seed, wtype):
    """wtype F16 = BASELINE configs[1] (Kokoro-82M fp16): the F16 GGUF's matrices and conv kernels
    (examples/quantize/quantize_impl.cpp:14-18), F16 mul_mats / convs / conv_transpose_1d with
    f16-rounded inputs on both sides."""
    cfg = ttship.kokoro_config(**dict(CFGS[name], weight_type=wtype, **({"max_tokens": 48, "max_total": 256} if n > 16 else {})))
    toks = tokens(n, seed)
    g = ttship.Kokoro(hip.iface(), cfg)
    o = ttship.Kokoro(py_oracle.iface(16), cfg)
    try:
        hg, lg = g.durations(toks)
        ho, lo = o.durations(toks)
        herr = float(np.max(np.abs(hg - ho)))
        print(f"kokoro {name} n={n} lengths {lo.astype(int).tolist()} hidden max err {herr:.3e}")
        assert np.array_equal(lg, lo), (lg, lo)
        assert herr <= 1e-3 * max(1.0, float(np.max(np.abs(ho))))
        total = int(lo.sum())
        rand = np.random.default_rng(seed + 7).random((cfg.gen.harmonic_num + 1, 600 * total), dtype=np.float32)
        pg = g.decode(toks, ho, lo, rand)
        po = o.decode(toks, ho, lo, rand)
        assert pg.shape == po.shape == (600 * total,)
        assert np.all(np.isfinite(pg))
        err = float(np.max(np.abs(pg.astype(np.float64) - po)))
        print(f"kokoro {name} total {total} frames pcm max err {err:.3e} (peak {float(np.max(np.abs(po))):.3f})")
        assert err <= 1e-4, f"max |pcm_gpu - pcm_oracle| = {err:.3e}"
        assert float(np.std(po)) > 1e-2
        # run() = durations() + decode() with the runner's own draws, deterministic across calls
        a = g.run(toks)
        b = g.decode(toks, hg, lg)
        assert np.array_equal(a, b) and np.array_equal(a, g.run(toks))
    finally:
        g.close()
        o.close()
