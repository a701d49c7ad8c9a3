"""Seeded sampler: the product's host restatement of sampler::sample (tts_sampler_sample,
tts.cpp_amd/csrc/sampler.cpp) against the independent Python oracle (oracle/py_sampler.py), over
the generation_configuration knobs (/root/reference/include/common.h:45-66: top_k, top_p,
temperature, repetition_penalty, sample) and several calls with the repetition state carried.
Bit-exact token ids are the bar."""
import numpy as np
import pytest

import py_sampler
import ttship

CONFIGS = [
    dict(),                                               # the defaults: top_k 50
    dict(top_k=1),
    dict(top_k=5, temperature=0.7),
    dict(top_k=0, top_p=0.9),                             # nucleus over the full sorted vocabulary
    dict(top_k=40, top_p=0.8, temperature=1.3),           # softmax first, top-k by probability, top-p
    dict(top_k=50, repetition_penalty=1.5),
    dict(top_k=0, top_p=0.95, repetition_penalty=1.2, temperature=0.9),
    dict(top_k=1088),                                     # top_k >= vocab: no nucleus
    dict(do_sample=0, repetition_penalty=1.3),            # sampler::max with the penalty
]


def logits_for(rng, NH, V, scale):
    x = (rng.standard_normal((NH, V)) * scale).astype(np.float32)
    x[:, rng.integers(0, V, 3)] += np.float32(4.0)  # a few peaked tokens, as trained heads have
    return x


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_host_sampler_matches_python_oracle(ci):
    kw = CONFIGS[ci]
    NH, V = 3, 257 if ci != 7 else 1088
    cfg = ttship.sampling(seed=1234 + ci, **kw)
    py = py_sampler.Sampler(NH, V, temperature=cfg.temperature, top_k=cfg.top_k, top_p=cfg.top_p,
                            repetition_penalty=cfg.repetition_penalty, do_sample=bool(cfg.do_sample), seed=cfg.seed)
    last = np.full(NH, -1, np.int32)
    count = np.zeros(NH, np.int32)
    rng = np.random.default_rng(ci)
    seen = set()
    for call in range(6):
        lg = logits_for(rng, NH, V, 1.0 + call * 0.5)
        if call >= 3:  # repeat the previous step's logits: the penalty state matters
            lg = prev
        cs = ttship.call_seed(cfg.seed, 2, call)
        assert cs == py_sampler.call_seed(cfg.seed, 2, call)
        got = ttship.host_sample(cfg, lg, cs, last, count)
        exp = py.sample(lg, stream=2, call=call)
        assert got.tolist() == exp, (call, got, exp)
        assert last.tolist() == (py.last if cfg.repetition_penalty != 1.0 else [-1] * NH)
        seen.update(got.tolist())
        prev = lg
    if kw.get("do_sample", 1) and kw.get("top_k", 50) != 1:
        assert len(seen) > NH  # it does sample


def test_call_seeds_distinct_and_in_range():
    s = {ttship.call_seed(7, b, c) for b in range(8) for c in range(64)}
    assert len(s) == 8 * 64 and min(s) >= 1 and max(s) <= 2147483646


def test_minstd_draws_match_libstdcxx():
    """py_sampler.MinStd restates std::uniform_real_distribution<float> over std::minstd_rand;
    the host sampler uses the library itself: with one head and top_k = V-1 over flat logits the
    token is the draw's position in the uniform CDF, so host == oracle pins the draw."""
    V = 1025
    cfg = ttship.sampling(top_k=V - 1, seed=99)
    flat = np.zeros((1, V), np.float32)
    for call in range(50):
        cs = ttship.call_seed(99, 0, call)
        u = py_sampler.MinStd(cs).uniform()
        tok = int(ttship.host_sample(cfg, flat, cs)[0])
        assert tok == py_sampler.Sampler(1, V, top_k=V - 1, seed=99).sample(flat, 0, call)[0]
        assert abs(tok / (V - 1) - float(u)) <= 2.0 / (V - 1)
