"""Host-side planning of the Parler decode step (no device): the fusion planner's coverage of the
reference node list (build_parler_graph, src/models/parler/model.cpp:520-614) built by the runner on
the oracle backend.  Every layer's cross-attention (n_enc <= 64 positions) must fold into the Q4_K
GEMV producing its query (TTS_FUSE_XATTN), the self-attention must be one fused item per layer."""
import numpy as np

import py_oracle
import ttship

TINY = dict(n_layers=3, hidden_size=256, n_attn_heads=4, ffn_size=1024, output_vocab=1088, max_ctx=96,
            prompt_vocab=512, max_positions=128)


def _decoded(batch):
    c = ttship.Parler(py_oracle.iface(2), ttship.parler_config(batch=batch, **TINY))
    prompt = (np.arange(6 * batch, dtype=np.int32).reshape(batch, 6) * 41) % 512
    c.prefill(prompt)
    c.decode(np.full((batch, 9), 7, dtype=np.int32))
    return c


def test_parler_step_plan_coverage():
    for batch in (1, 3):
        c = _decoded(batch)
        st = c.plan_stats()
        L = TINY["n_layers"]
        assert st["attn"] == 2 * L, st          # self + cross per layer
        assert st["xattn"] == L, st             # every cross-attention rides its query GEMV
        without = c.plan_stats(ttship.FUSE_ALL & ~ttship.FUSE["XATTN"])
        assert without["xattn"] == 0 and without["attn"] == 2 * L
        # the reference's node order (parler_build_kv_store expands K / V first, Q at the attention):
        # q / k / v still one launch per layer, the K / V cache stores in its epilogue
        assert st["gemv_max_group"] >= 3, st
        assert st["gemv"] == 6 * L + 1, st     # qkv, o, cross-q (+ cross-attention), cross-o, fc1, fc2; heads
        c.close()


def test_parler_node_order_is_the_reference_order():
    """build_parler_graph's order: LN, K, its cache view and CPY, V, transpose, cont, view, CPY, ...,
    then Q (model.cpp:544-548 with parler_build_kv_store :420-439): no reordering in the runner."""
    c = _decoded(1)
    try:
        names = [c.node(i, cap=4)[0] for i in range(c.last_graph_nodes())]
        mm = [i for i, o in enumerate(names) if o == "MUL_MAT"]
        first_layer = names[mm[0]:mm[0] + 12]
        assert first_layer[:4] == ["MUL_MAT", "VIEW", "CPY", "MUL_MAT"], first_layer
        assert "TRANSPOSE" in first_layer and first_layer.count("CPY") == 2
    finally:
        c.close()


def _ragged_prompts(lens, vocab=512):
    return [((np.arange(L, dtype=np.int32) * (31 + 2 * r) + 5 * r + 1) % vocab).astype(np.int32) for r, L in enumerate(lens)]


def test_ragged_batch_equals_each_prompt_alone():
    """A ragged lock-step batch (tts_parler_prefill_ragged: prompts of 5, 9 and 7 tokens in one prompt
    pass, then decoded in lockstep at their own positions, each with its own mask over the padding
    slots) gives every prompt the tokens of its own B = 1 run, on the oracle."""
    lens = [5, 9, 7]
    prompts = _ragged_prompts(lens)
    c = ttship.Parler(py_oracle.iface(4), ttship.parler_config(batch=3, **TINY))
    c.prefill_ragged(prompts)
    got = c.generate(8)
    c.close()
    for r, p in enumerate(prompts):
        a = ttship.Parler(py_oracle.iface(4), ttship.parler_config(batch=1, **TINY))
        a.prefill(p.reshape(1, -1))
        ref = a.generate(8)
        a.close()
        assert np.array_equal(got[r], ref[0]), f"prompt {r}"


def test_ragged_batch_rejects_bad_lengths():
    c = ttship.Parler(py_oracle.iface(2), ttship.parler_config(batch=2, **TINY))
    try:
        import pytest
        with pytest.raises(RuntimeError):
            c.prefill_ragged([np.zeros(0, np.int32), np.ones(3, np.int32)])  # an empty prompt
        c.prefill_ragged(_ragged_prompts([3, 4]))
        with pytest.raises(RuntimeError):
            c.prefill_ragged(_ragged_prompts([3, 4]))  # only from an empty cache
    finally:
        c.close()
