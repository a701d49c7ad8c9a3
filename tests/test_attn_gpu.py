"""Fused decode attention vs the oracle running the reference's unfused node chain
(Parler model.cpp:549-571): cont(K view) -> mul_mat(K, q) -> soft_max_ext(mask, 1/sqrt(hd)) ->
mul_mat(kq, V view) -> permute(2, 0, 1, 3) -> cont, with K / V read from cache layouts.

Kernel choice depends on the context length (k_attn.hip): P <= 64 -> k_attn_small (sequential
sums, bit-exact); P >= TTS_HIP_OPT_ATTN_FUSED (default off) -> k_attn_fused (one 1024-thread launch);
otherwise P >= TTS_HIP_OPT_ATTN_SPLIT (default 128) -> k_attn_scores + k_attn_pv (split over
positions, then over output dims); otherwise k_attn_decode_rows with V prefetched (P <= 512) or
streamed; hd 128 (Dia / Orpheus head size).  `mode` runs every case through each kernel.  The row
kernels reassociate the f64 sums (quad / row DPP reductions), so they are held to <= 1 ulp with almost
all elements exact; the fused kernel runs the row kernel's sums in its order, so it is bit-identical
to it.
"""
import numpy as np
import pytest

import audio_ops as ao
import nodes as nd
import ttship

F32 = ttship.F32


def build(g, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx):
    """q (B, H, hd); kc (B, P_cap, Hk*hd) position-major K cache; vc (B, Hk*hd, max_ctx) transposed V."""
    ql = g.leaf(q.reshape(B, 1, H, hd))                       # ne [hd, H, 1, B]
    qp = g.permute(ql, (0, 2, 1, 3))                          # [hd, 1, H, B]
    qc = g.node("CONT", F32, [hd, 1, H, B], [qp])
    kl = g.leaf(kc)                                           # ne [Hk*hd, P_cap, B]
    k = g.view(kl, [hd, P, Hk, B], [4, Hk * hd * 4, hd * 4, kl.nb[2]])
    kcont = g.node("CONT", F32, [hd, P, Hk, B], [k])
    kq = g.node("MUL_MAT", F32, [P, 1, H, B], [kcont, qc])
    ml = g.leaf(mask.reshape(1, P))
    sm = g.node("SOFT_MAX", F32, [P, 1, H, B], [kq, ml], fparams={0: float(1.0 / np.sqrt(hd)), 1: 0.0})
    vl = g.leaf(vc)                                           # ne [max_ctx, Hk*hd, B]
    v = g.view(vl, [P, hd, Hk, B], [4, max_ctx * 4, max_ctx * hd * 4, vl.nb[2]])
    kqv = g.node("MUL_MAT", F32, [1, hd, H, B], [sm, v])
    merged = g.permute(kqv, (2, 0, 1, 3))                     # [hd, H, 1, B]
    return g.node("CONT", F32, [hd, H, 1, B], [merged])


@pytest.mark.gpu
@pytest.mark.parametrize("P,hd,H,Hk,B", [(3, 64, 16, 16, 2), (64, 64, 16, 16, 1), (65, 64, 4, 4, 1), (500, 64, 16, 16, 2),
                                         (700, 64, 16, 16, 1), (1024, 64, 4, 4, 1), (1500, 64, 4, 4, 1),
                                         (37, 128, 16, 16, 2), (430, 128, 8, 8, 1), (1, 64, 4, 4, 1),
                                         (1309, 64, 16, 16, 8), (2100, 128, 24, 24, 1), (128, 64, 16, 16, 3),
                                         (257, 128, 16, 16, 2), (4096, 64, 16, 16, 2)])
@pytest.mark.parametrize("mode", ["fused", "split", "split_ks1", "split_ks4_pv8", "rows"])
def test_fused_attention_matches_unfused_chain(hip, P, hd, H, Hk, B, mode):
    set_mode(hip, mode)
    rng = np.random.default_rng(P * 7 + hd)
    max_ctx = P + 40
    q = rng.standard_normal((B, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, Hk * hd)).astype(np.float32)
    vc = rng.standard_normal((B, Hk * hd, max_ctx)).astype(np.float32)
    mask = np.zeros(P, np.float32)
    if P > 4:
        mask[P // 3] = -np.inf  # a masked key inside the window
    g1, g2 = nd.Graph(), nd.Graph()
    o1 = build(g1, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    o2 = build(g2, q, kc, vc, mask, P, hd, H, Hk, B, max_ctx)
    g1.run_hip(hip)
    g2.run_oracle(n_threads=8)
    set_mode(hip, "default")
    gpu, ref = g1.node_array(o1), g2.node_array(o2)
    if P <= 64:
        assert np.array_equal(gpu, ref)
    else:
        assert ao.ulp_diff(gpu, ref) <= 1 and np.mean(gpu != ref) <= 1e-3


def set_mode(hip, mode):
    """split_ks1 / split_ks4_pv8: the split pair with 128 / 512 positions per scores workgroup and 8
    output dims per P.V workgroup (TTS_HIP_OPT_ATTN_KS / _PV8); the same sums per element."""
    split = mode.startswith("split") or mode == "default"
    hip.set_option(ttship.OPT["ATTN_FUSED"], ttship.ATTN_FUSED_ON if mode == "fused" else 0)
    hip.set_option(ttship.OPT["ATTN_SPLIT"], ttship.ATTN_SPLIT_DEFAULT if split else 0)
    hip.set_option(ttship.OPT["ATTN_KS"], 1 if mode == "split_ks1" else 4 if mode == "split_ks4_pv8" else 2)
    hip.set_option(ttship.OPT["ATTN_PV8"], 1 if mode == "split_ks4_pv8" else 0)
    hip.set_option(ttship.OPT["ATTN_PV_MP"], 0 if mode in ("split_ks4_pv8", "split_pv16") else 2 if mode == "split_mp8" else 1)


@pytest.mark.gpu
@pytest.mark.parametrize("P,hd,B", [(129, 64, 3), (460, 64, 5), (512, 64, 2), (513, 64, 2), (300, 128, 2),
                                   (1024, 64, 16), (1309, 64, 16), (1100, 128, 16), (4096, 64, 16), (1309, 64, 4)])
def test_pv_all_dims_bit_identical(hip, P, hd, B):
    """The split P.V with every dim of a (head, query, sequence) in one workgroup (k_attn_pv_mp, any context: items
    of 512 positions; the softmax once per head; past 512 keys only with >= 256 rows, so B = 16 there) against 16 dims per
    workgroup (k_attn_pv): the same sums, identical bits."""
    H = 16
    rng = np.random.default_rng(P * 3 + hd + B)
    max_ctx = (P + 8 + 3) // 4 * 4  # 16-B V rows: the vector-load P.V kernels
    q = rng.standard_normal((B, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, H * hd)).astype(np.float32)
    vc = rng.standard_normal((B, H * hd, max_ctx)).astype(np.float32)
    mask = np.zeros(P, np.float32)
    mask[P // 2] = -np.inf
    outs = []
    for mode in ("split", "split_pv16", "split_mp8"):
        set_mode(hip, mode)
        g = nd.Graph()
        o = build(g, q, kc, vc, mask, P, hd, H, H, B, max_ctx)
        g.run_hip(hip)
        outs.append(g.node_array(o))
    set_mode(hip, "default")
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


@pytest.mark.gpu
@pytest.mark.parametrize("P,hd,B", [(129, 64, 2), (880, 64, 8), (1309, 64, 4), (3000, 64, 1), (700, 128, 2), (2100, 128, 1)])
def test_fused_attention_bit_identical_to_row_kernel(hip, P, hd, B):
    """k_attn_fused runs k_attn_decode_rows' f64 sums in the same order: identical bits."""
    H = 16
    rng = np.random.default_rng(P + hd)
    max_ctx = P + 8
    q = rng.standard_normal((B, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, H * hd)).astype(np.float32)
    vc = rng.standard_normal((B, H * hd, max_ctx)).astype(np.float32)
    mask = np.zeros(P, np.float32)
    mask[P // 2] = -np.inf
    outs = []
    for mode in ("fused", "rows"):
        set_mode(hip, mode)
        g = nd.Graph()
        o = build(g, q, kc, vc, mask, P, hd, H, H, B, max_ctx)
        g.run_hip(hip)
        outs.append(g.node_array(o))
    set_mode(hip, "default")
    assert np.array_equal(outs[0], outs[1])


def build_multi(g, q, kc, vc, mask, P, n, hd, H, Hk, B, max_ctx):
    """n queries per sequence (a prompt pass): q (B, n, H, hd), mask [n, P]; otherwise as build()."""
    ql = g.leaf(q)                                            # ne [hd, H, n, B]
    qp = g.permute(ql, (0, 2, 1, 3))                          # [hd, n, H, B]
    qc = g.node("CONT", F32, [hd, n, H, B], [qp])
    kl = g.leaf(kc)
    k = g.view(kl, [hd, P, Hk, B], [4, Hk * hd * 4, hd * 4, kl.nb[2]])
    kcont = g.node("CONT", F32, [hd, P, Hk, B], [k])
    kq = g.node("MUL_MAT", F32, [P, n, H, B], [kcont, qc])
    ml = g.leaf(mask)                                         # ne [P, n]
    sm = g.node("SOFT_MAX", F32, [P, n, H, B], [kq, ml], fparams={0: float(1.0 / np.sqrt(hd)), 1: 0.0})
    vl = g.leaf(vc)
    v = g.view(vl, [P, hd, Hk, B], [4, max_ctx * 4, max_ctx * hd * 4, vl.nb[2]])
    kqv = g.node("MUL_MAT", F32, [n, hd, H, B], [sm, v])
    merged = g.permute(kqv, (2, 0, 1, 3))                     # [hd, H, n, B]
    return g.node("CONT", F32, [hd, H, n, B], [merged])


@pytest.mark.gpu
@pytest.mark.parametrize("P,n,hd,H,Hk,B", [(18, 18, 64, 16, 16, 4), (3, 18, 64, 16, 16, 2), (64, 64, 64, 4, 4, 2),
                                           (37, 5, 128, 8, 8, 2), (9, 4, 64, 16, 16, 3), (1, 4, 64, 4, 4, 1)])
def test_short_context_many_queries_bit_exact(hip, P, n, hd, H, Hk, B):
    """A prompt pass's short-context attention (n >= 4 queries, P <= 64: k_attn_small_q, K / V staged in LDS
    once per head and sequence): bit-identical to the oracle's unfused chain, causal mask included."""
    rng = np.random.default_rng(P * 13 + n + hd)
    max_ctx = P + 24
    q = rng.standard_normal((B, n, H, hd)).astype(np.float32)
    kc = rng.standard_normal((B, max_ctx, Hk * hd)).astype(np.float32)
    vc = rng.standard_normal((B, Hk * hd, max_ctx)).astype(np.float32)
    mask = np.zeros((n, P), np.float32)
    for i in range(n):  # causal over the last n positions (the prompt's own rows)
        mask[i, max(0, P - n) + i + 1:] = -np.inf
    g1, g2 = nd.Graph(), nd.Graph()
    o1 = build_multi(g1, q, kc, vc, mask, P, n, hd, H, Hk, B, max_ctx)
    o2 = build_multi(g2, q, kc, vc, mask, P, n, hd, H, Hk, B, max_ctx)
    g1.run_hip(hip)
    g2.run_oracle(n_threads=8)
    gpu, ref = g1.node_array(o1), g2.node_array(o2)
    assert np.array_equal(gpu, ref)
