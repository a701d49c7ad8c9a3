"""Orpheus-3B decoder parity: the HIP backend vs the CPU oracle on the same graph
(build_orpheus_graph, src/models/orpheus/model.cpp:230-311).

Bars (BASELINE.json north_star): greedy (sampler::max) token ids bit-exact; logits within
1e-4 * max|logit| + 1e-4 (the only f32 differences are reduction orders outside ggml's exact paths).
"""
import numpy as np
import pytest

import py_oracle
import ttship

TINY = dict(n_layers=2, hidden_size=256, n_attn_heads=4, n_kv_attn_heads=2, head_size=64, ffn_size=512,
            vocab_size=1000, max_ctx=48)
# real Orpheus widths (3072 / 24 x 128 / 8 KV heads / 8192 / 156 940 vocab), two layers
WIDE = dict(n_layers=2, max_ctx=32)


def run_pair(hip, cfg_kw, batch, n_prompt, n_gen, tile_bytes=None, mask=None, expect=None):
    if tile_bytes is not None:
        hip.set_option(ttship.OPT["Q4K_TILE_BYTES"], tile_bytes)
    try:
        g = ttship.Orpheus(hip.iface(), ttship.orpheus_config(batch=batch, **cfg_kw))
    finally:
        hip.set_option(ttship.OPT["Q4K_TILE_BYTES"], 4 << 20)
    if mask is not None:
        hip.set_option(ttship.OPT["FUSION"], mask)
    try:
        _run_pair(g, cfg_kw, batch, n_prompt, n_gen, expect, ttship.FUSE_ALL if mask is None else mask)
    finally:
        hip.set_option(ttship.OPT["FUSION"], ttship.FUSE_ALL)


def _run_pair(g, cfg_kw, batch, n_prompt, n_gen, expect, mask):
    c = ttship.Orpheus(py_oracle.iface(16), ttship.orpheus_config(batch=batch, **cfg_kw))
    try:
        V = c.cfg.vocab_size
        prompt = (np.arange(n_prompt * batch, dtype=np.int32).reshape(batch, n_prompt) * 7919 + 3) % V
        lg, lc = g.prefill(prompt), c.prefill(prompt)
        tol = 1e-4 * np.abs(lc).max() + 1e-4
        assert np.abs(lg - lc).max() <= tol, np.abs(lg - lc).max()
        first = lc.argmax(axis=1).astype(np.int32)
        assert np.array_equal(lg.argmax(axis=1), first)
        tg, tc = g.generate(first, n_gen), c.generate(first, n_gen)
        assert np.array_equal(tg, tc), f"token mismatch\n{tg}\n{tc}"
        dg, dc = g.decode(tg[:, -1]), c.decode(tc[:, -1])
        assert np.abs(dg - dc).max() <= 1e-4 * np.abs(dc).max() + 1e-4
        if expect:
            st = g.plan_stats(mask)
            for k, v in expect.items():
                assert st[k] == v, f"plan {k}: {st[k]} != {v} ({st})"
    finally:
        g.close()
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
def test_orpheus_tiny(hip, batch):
    run_pair(hip, TINY, batch, 6, 10)


@pytest.mark.gpu
def test_orpheus_tiny_all_tiled(hip):
    """Every Q4_K matrix (embedding and head included) in the tile layout: matrix-core GEMVs."""
    run_pair(hip, TINY, 2, 5, 8, tile_bytes=1)


@pytest.mark.gpu
def test_orpheus_wide_two_layers(hip):
    """Full Orpheus widths (tile-layout GEMVs for q/o/gate/up/down and the 156 940-row head)."""
    run_pair(hip, WIDE, 2, 4, 3)


@pytest.mark.gpu
def test_orpheus_3b_full_depth(hip):
    """BASELINE configs[4] at full depth: Orpheus-3B's 28 layers and the 156 940-row Q4_K head
    (src/models/orpheus/model.h:31-46, model.cpp:230-311), 2 prompts, 16 greedy steps: tokens bit-exact,
    logits within 1e-4 -- the K-relay chains, tile-layout head and GQA cache copies over every layer."""
    run_pair(hip, dict(max_ctx=40), 2, 4, 16)


@pytest.mark.gpu
def test_orpheus_wide_batch8(hip):
    """The bench's shape (8 prompts = 8 GEMV columns): q / k / v as one launch over the stored-tiled q
    and the tile-layout copies of k / v, the SwiGLU launch, residue-split tiles; one GEMV item per
    (qkv, o, SwiGLU, down) and layer plus the head -- in the reference's node order (K's rope and cache
    copies, then V, then Q), Q hoisted into the K / V launch (through scratch when the allocator gave it
    K's memory)."""
    run_pair(hip, WIDE, 8, 2, 2, expect={"gemv": 4 * WIDE["n_layers"] + 1, "gemv_max_group": 3})


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["mf", "inkernel", "kr_inkernel"])
def test_orpheus_wide_batch8_gemv_paths(hip, path):
    """The bench shape on the older matrix-core paths: k_gemv_q4K_mf after the quantize pass (K relay
    off), and every workgroup quantizing its own operands (quantize pass off); tokens bit-exact either way
    (the default, K relay after the pass, is test_orpheus_wide_batch8)."""
    if path == "kr_inkernel":  # the K relay with the prologue in every workgroup (K <= 4096)
        hip.set_option(ttship.OPT["GEMV_KR_INKERNEL"], 4096)
        try:
            run_pair(hip, WIDE, 8, 2, 2)
        finally:
            hip.set_option(ttship.OPT["GEMV_KR_INKERNEL"], 0)
        return
    opt = "GEMV_KRELAY" if path == "mf" else "GEMV_PREQUANT"
    hip.set_option(ttship.OPT[opt], 0)
    try:
        run_pair(hip, WIDE, 8, 2, 2)
    finally:
        hip.set_option(ttship.OPT[opt], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("drop", ["none", "EPI", "CONTREAD", "MCPY", "GROUP"])
def test_orpheus_tiny_tiled_fusion_masks(hip, drop):
    """All matrices tiled at 8 columns (SwiGLU epilogue, residue split, mixed-row q / k / v groups) with
    each related fusion pattern switched off in turn: tokens bit-exact, logits within the bar."""
    mask = ttship.FUSE_ALL if drop == "none" else ttship.FUSE_ALL & ~ttship.FUSE[drop]
    run_pair(hip, TINY, 8, 4, 6, tile_bytes=1, mask=mask)


@pytest.mark.gpu
def test_orpheus_hd128_mid_context(hip):
    """head_size 128 at 65..127 keys: the row attention kernel over Orpheus' strided (transposed-view) V
    with every V value requested before the softmax."""
    cfg = dict(n_layers=1, hidden_size=512, n_attn_heads=4, n_kv_attn_heads=2, head_size=128, ffn_size=512,
               vocab_size=1000, max_ctx=160)
    run_pair(hip, cfg, 3, 70, 12)
