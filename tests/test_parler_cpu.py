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
