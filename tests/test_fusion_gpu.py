"""graph_compute fusion must not change a single bit: every fusion pattern alone and all together,
on the Parler step graph (B=1 = the reference's node list, B=3 = lockstep batch), against the oracle.
"""
import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=96,
            prompt_vocab=512, max_positions=128)
MASKS = {"off": 0, "ln": 1, "group": 2, "kv": 2 | 4, "epi": 8, "heads": 16, "attn": 32, "embed": 256,
         "xattn": 32 | 2048, "ln_xattn": 1 | 32 | 2048, "all_but_xattn": ttship.FUSE_ALL & ~2048, "all": ttship.FUSE_ALL}


@pytest.fixture(scope="module")
def oracle_runs():
    out = {}
    for batch in (1, 3):
        c = ttship.Parler(py_oracle.iface(8), ttship.parler_config(batch=batch, **TINY))
        prompt = (np.arange(6 * batch, dtype=np.int32).reshape(batch, 6) * 41) % 512
        c.prefill(prompt)
        toks = c.generate(5)
        logits = c.decode(np.full((batch, 9), 7, dtype=np.int32))
        c.close()
        out[batch] = (prompt, toks, logits)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
@pytest.mark.parametrize("name", list(MASKS))
def test_fusion_bit_exact(hip, oracle_runs, batch, name):
    prompt, toks_ref, logits_ref = oracle_runs[batch]
    hip.set_option(0, MASKS[name])
    try:
        g = ttship.Parler(hip.iface(), ttship.parler_config(batch=batch, **TINY))
        g.prefill(prompt)
        toks = g.generate(5)
        logits = g.decode(np.full((batch, 9), 7, dtype=np.int32))
        g.close()
    finally:
        hip.set_option(0, ttship.FUSE_ALL)
    assert np.array_equal(toks, toks_ref), f"{name}: tokens differ\n{toks}\n{toks_ref}"
    diff = np.abs(logits.astype(np.float64) - logits_ref)
    assert np.array_equal(logits.view(np.uint32), logits_ref.view(np.uint32)), f"{name}: max |dlogit| {diff.max()}"
