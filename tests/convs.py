"""Node-list builders for the codec convolutions (shared by the oracle-vs-torch and HIP-vs-oracle
tests): ggml_conv_1d = IM2COL(F16) -> MUL_MAT, and the fork's CONV_TRANSPOSE_1D."""
import numpy as np

import ttship

F32, F16 = ttship.F32, ttship.F16


def conv_transpose_1d(g, x, w, s, p, d, op, grp, wtype=F32):
    """x: (IC, L) f32, w: torch layout (IC, OC/g, K) -> node [OL, OC]; wtype F16: an F16 kernel
    (Kokoro's F16 GGUF), whose product rounds the input to f16."""
    IC, L = x.shape
    K = w.shape[2]
    OC = w.shape[1] * grp
    OL = (L - 1) * s - 2 * p + d * (K - 1) + op + 1
    wl = g.leaf(w.astype(np.float16) if wtype == F16 else w, typ=wtype)
    return g.node("CONV_TRANSPOSE_1D", F32, [OL, OC], [wl, g.leaf(x)], params=[s, p, d, op, grp])


def conv_1d(g, x, w, s, p, d, wtype=F32):
    """ggml_conv_1d: x (IC, L) f32, w (OC, IC, K) -> node [OL, OC] (= mul_mat of the F16 im2col)."""
    IC, L = x.shape
    OC, _, K = w.shape
    OL = (L + 2 * p - d * (K - 1) - 1) // s + 1
    wl = g.leaf(w.astype(np.float16) if wtype == F16 else w, typ=wtype)
    col = g.node("IM2COL", F16, [IC * K, OL, 1], [wl, g.leaf(x)], params=[s, 1, p, 0, d, 1, 0])
    col2 = g.view(col, [IC * K, OL, 1, 1], [2, 2 * IC * K, 2 * IC * K * OL, 2 * IC * K * OL], op="RESHAPE")
    es = 2 if wtype == F16 else 4
    w2 = g.view(wl, [K * IC, OC, 1, 1], [es, es * K * IC, es * K * IC * OC, es * K * IC * OC], op="RESHAPE")
    return g.node("MUL_MAT", F32, [OL, OC], [col2, w2])


def ref_conv_transpose_1d(x, w, s, p, d, op, grp):
    """float64 numpy restatement (PyTorch semantics), for shapes too large to keep as fixtures."""
    IC, L = x.shape
    _, OCg, K = w.shape
    OC = OCg * grp
    OL = (L - 1) * s - 2 * p + d * (K - 1) + op + 1
    y = np.zeros((OC, OL), dtype=np.float64)
    ICg = IC // grp
    for ic in range(IC):
        gi = ic // ICg
        for k in range(K):
            o = np.arange(L) * s - p + k * d
            ok = (o >= 0) & (o < OL)
            for ocl in range(OCg):
                y[gi * OCg + ocl, o[ok]] += x[ic, ok].astype(np.float64) * float(w[ic, ocl, k])
    return y
