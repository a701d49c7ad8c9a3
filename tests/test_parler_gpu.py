"""End-to-end Parler decoder parity: the HIP backend vs the CPU oracle on the same graph.

Bars (BASELINE.json north_star): greedy (sampler::max) token ids bit-exact at fixed seed;
logits within 1e-4 * max|logit| + 1e-4 (f32 reduction order is the only difference).
"""
import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=128,
            prompt_vocab=512, max_positions=160)


def make_pair(hip, **kw):
    cfg = ttship.parler_config(**kw)
    g = ttship.Parler(hip.iface(), cfg)
    c = ttship.Parler(py_oracle.iface(8), ttship.parler_config(**kw))
    return g, c


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
def test_tiny_tokens_and_logits(hip, batch):
    g, c = make_pair(hip, batch=batch, **TINY)
    try:
        prompt = (np.arange(7 * batch, dtype=np.int32).reshape(batch, 7) * 37) % 512
        g.prefill(prompt)
        c.prefill(prompt)
        tg = g.generate(12)
        tc = c.generate(12)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
        toks = np.full((batch, 9), 5, dtype=np.int32)
        lg = g.decode(toks)
        lc = c.decode(toks)
        tol = 1e-4 * np.abs(lc).max() + 1e-4
        assert np.abs(lg - lc).max() <= tol, np.abs(lg - lc).max()
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
def test_full_parler_mini_q4k_tokens(hip):
    """Full Parler-mini shapes (24 layers, d=1024, Q4_K), batch 2, 6 greedy steps."""
    g, c = make_pair(hip, batch=2)
    try:
        prompt = np.array([[11, 29, 400, 7, 1, 3000, 16], [5, 6, 7, 8, 9, 10, 11]], dtype=np.int32)
        g.prefill(prompt)
        c.prefill(prompt)
        tg = g.generate(6)
        tc = c.generate(6)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
    finally:
        g.close()
        c.close()
