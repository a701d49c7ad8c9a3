"""Device sampler (tts_hip_sample_step, k_sample.hip) vs the host sampler (tts_sampler_sample, itself
pinned to oracle/py_sampler.py by tests/test_sampler_cpu.py): bit-identical tokens, repetition state
and next-token rule over Parler / Dia / Orpheus vocabularies and the sampler knobs."""
import numpy as np
import pytest

import ttship

CASES = [  # B, NH, V, sampling kwargs
    (4, 9, 1088, dict()),                                   # Parler, defaults (top_k 50)
    (2, 9, 1028, dict(top_k=5, temperature=0.7)),           # Dia
    (3, 9, 1088, dict(top_k=0, top_p=0.9)),
    (2, 9, 1088, dict(top_k=40, top_p=0.8, temperature=1.3)),
    (2, 9, 1088, dict(top_k=50, repetition_penalty=1.5)),
    (2, 9, 1028, dict(top_k=0, top_p=0.95, repetition_penalty=1.2, temperature=0.9)),
    (2, 9, 1088, dict(top_k=0)),                            # softmax over the whole vocabulary
    (2, 9, 1088, dict(do_sample=0, repetition_penalty=1.3)),
    (3, 1, 156940, dict()),                                 # Orpheus: wide vocabulary, top_k 50
    (2, 1, 156940, dict(top_k=64, temperature=0.8, repetition_penalty=1.1)),
    (2, 1, 156940, dict(do_sample=0)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_device_sampler_matches_host(hip, ci):
    B, NH, V, kw = CASES[ci]
    cfg = ttship.sampling(seed=77 + ci, **kw)
    rng = np.random.default_rng(ci)
    rep = np.tile(np.array([-1, 0], np.int32), B * NH)
    last = np.full((B, NH), -1, np.int32)
    count = np.zeros((B, NH), np.int32)
    seen = np.zeros(B * NH, np.int32)
    lg = None
    for call in range(4):
        if call != 2:  # call 2 repeats call 1's logits (the penalty state matters)
            lg = (rng.standard_normal((B, NH, V)) * (1.0 + call)).astype(np.float32)
            lg[:, :, rng.integers(0, V, 4)] += np.float32(3.0)
        hist, nxt, seen, rep = hip.sample_step(lg, cfg, call, rep, step=call + 20, eos=int(lg.shape[2] - 1), eos_seen=seen)
        for b in range(B):
            exp = ttship.host_sample(cfg, lg[b], ttship.call_seed(cfg.seed, b, call), last[b], count[b])
            assert hist[b].tolist() == exp.tolist(), (call, b, hist[b], exp)
            assert np.array_equal(nxt[:, b], np.where(seen.reshape(B, NH)[b] != 0, V - 1, exp))
        if cfg.repetition_penalty != 1.0:
            assert np.array_equal(rep.reshape(B * NH, 2)[:, 0], last.reshape(-1))
            assert np.array_equal(rep.reshape(B * NH, 2)[:, 1], count.reshape(-1))


@pytest.mark.gpu
def test_device_sampler_wide_rejects_unsupported(hip):
    lg = np.zeros((1, 1, 156940), np.float32)
    with pytest.raises(RuntimeError):
        hip.sample_step(lg, ttship.sampling(top_k=0, top_p=0.9), 0)
