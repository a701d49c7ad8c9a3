"""Orpheus-3B runner on the CPU oracle (no device): graph shape of build_orpheus_graph
(src/models/orpheus/model.cpp:230-311) with the repeat-interleaved KV store (:194-228), determinism
of the greedy loop, prefill-then-decode consistency, and the fusion planner's view of the step."""
import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, n_kv_attn_heads=2, head_size=64, ffn_size=512,
            vocab_size=1000, max_ctx=48)


def test_rope_factors_follow_llama3_scaling():
    # orpheus_gguf_encoder.prepare_rope_frequencies: 1 for short wavelengths, `factor` for long ones
    c = ttship.Orpheus(py_oracle.iface(2), ttship.orpheus_config(**TINY))
    try:
        assert c.weight_bytes() > 0
    finally:
        c.close()


@pytest.mark.parametrize("batch", [1, 2])
def test_orpheus_tiny_greedy_deterministic(batch):
    outs = []
    for _ in range(2):
        c = ttship.Orpheus(py_oracle.iface(4), ttship.orpheus_config(batch=batch, **TINY))
        try:
            prompt = (np.arange(5 * batch, dtype=np.int32).reshape(batch, 5) * 37) % 1000
            lg = c.prefill(prompt)
            first = lg.argmax(axis=1).astype(np.int32)
            toks = c.generate(first, 6)
            assert c.position() == 5 + 6
            outs.append(toks)
        finally:
            c.close()
    assert np.array_equal(outs[0], outs[1])
    assert outs[0].shape == (batch, 6)


def test_orpheus_batch_rows_match_single_prompts():
    """Lockstep batching: prompt b of a batch-2 runner decodes exactly as a batch-1 runner."""
    prompts = (np.arange(10, dtype=np.int32).reshape(2, 5) * 53 + 11) % 1000
    cb = ttship.Orpheus(py_oracle.iface(4), ttship.orpheus_config(batch=2, **TINY))
    try:
        lb = cb.prefill(prompts)
        tb = cb.generate(lb.argmax(axis=1).astype(np.int32), 4)
    finally:
        cb.close()
    for b in range(2):
        c1 = ttship.Orpheus(py_oracle.iface(4), ttship.orpheus_config(batch=1, **TINY))
        try:
            l1 = c1.prefill(prompts[b:b + 1])
            assert np.array_equal(l1[0], lb[b])
            t1 = c1.generate(l1.argmax(axis=1).astype(np.int32), 4)
            assert np.array_equal(t1[0], tb[b])
        finally:
            c1.close()


def test_orpheus_step_plan():
    c = ttship.Orpheus(py_oracle.iface(2), ttship.orpheus_config(**TINY))
    try:
        c.prefill(np.arange(4, dtype=np.int32)[None])
        c.decode(np.array([7], dtype=np.int32))
        assert c.last_graph_nodes() > 20 * TINY["n_layers"]
        st = c.plan_stats()
        L = TINY["n_layers"]
        assert st["attn"] == L, st   # transposed-V cont folded: one fused attention per layer
        # K: rope + its repeat-interleave copies as one pass; V: written into its copies by the GEMV
        assert st["mcpy"] == L, st
        assert st["ln"] + st["gemv"] >= 5 * L, st
    finally:
        c.close()
