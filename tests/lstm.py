"""Node-list builder restating Kokoro's unrolled LSTM (build_lstm / build_lstm_run,
src/models/kokoro/model.cpp:35-86) node for node, plus a float64 numpy restatement of
torch.nn.LSTM (gate order i, f, g, o) that pins the graph's semantics."""
import numpy as np

import ttship

F32, F16 = ttship.F32, ttship.F16
UN_TANH, UN_SIGMOID = 2, 4


def lstm_weights(seed, n_in, hd, scale=0.15, bidirectional=True):
    """torch nn.LSTM-layout weights per direction: w_ih [4H, in], w_hh [4H, H], b_ih, b_hh [4H]."""
    rng = np.random.default_rng(seed)
    dirs = []
    for _ in range(2 if bidirectional else 1):
        dirs.append({k: (rng.standard_normal(s) * scale).astype(np.float32) for k, s in
                     (("w_ih", (4 * hd, n_in)), ("w_hh", (4 * hd, hd)), ("b_ih", (4 * hd,)), ("b_hh", (4 * hd,)))})
    return dirs


def _mm(g, w, x, ne):
    return g.node("MUL_MAT", F32, ne, [w, x])


def lstm_run(g, x, h0, c0, d, reversed_=False, wtype=F32):
    """build_lstm_run: x node [n_in, T]; d = one direction's weights.  Returns the outputs node
    [H, T] (concat chain), and the final h / c nodes."""
    hd = d["w_hh"].shape[1]
    T = x.ne[1]
    ws, bs = [], []
    for gi in range(4):  # the reference's weights[0..7] / biases[0..7]: (ih, hh) per gate i, f, g, o
        for key, bkey in (("w_ih", "b_ih"), ("w_hh", "b_hh")):
            w = d[key][gi * hd:(gi + 1) * hd]
            ws.append(g.leaf(w.astype(np.float16), typ=F16) if wtype == F16 else g.leaf(w))
            bs.append(g.leaf(d[bkey][gi * hd:(gi + 1) * hd]))
    pre = []
    for gi in range(4):
        m = _mm(g, ws[2 * gi], x, [hd, T])
        pre.append(g.node("ADD", F32, [hd, T], [m, bs[2 * gi]]))
    h, c, outputs = h0, c0, None
    for index in range(T):
        i = T - 1 - index if reversed_ else index
        gates = []
        for gi, uop in enumerate((UN_SIGMOID, UN_SIGMOID, UN_TANH, UN_SIGMOID)):
            P = pre[gi]
            cur = g.view(P, [hd, 1, 1, 1], [4, P.nb[1], P.nb[2], P.nb[3]], offs=P.nb[1] * i)
            mm = _mm(g, ws[2 * gi + 1], h, [hd, 1])
            ab = g.node("ADD", F32, [hd, 1], [mm, bs[2 * gi + 1]])
            ap = g.node("ADD", F32, [hd, 1], [cur, ab])
            gates.append(g.node("UNARY", F32, [hd, 1], [ap], params=[uop]))
        I, Fg, G, O = gates
        fc = g.node("MUL", F32, [hd, 1], [Fg, c])
        ig = g.node("MUL", F32, [hd, 1], [I, G])
        c = g.node("ADD", F32, [hd, 1], [fc, ig])
        th = g.node("UNARY", F32, [hd, 1], [c], params=[UN_TANH])
        h = g.node("MUL", F32, [hd, 1], [th, O])
        if index == 0:
            outputs = h
        else:
            srcs = [h, outputs] if reversed_ else [outputs, h]
            outputs = g.node("CONCAT", F32, [hd, index + 1], srcs, params=[1])
    return outputs, h, c


def lstm(g, x_arr, dirs, wtype=F32, h0=None, c0=None):
    """build_lstm for one cell: forward run, reverse run (bidirectional), concat along dim 0."""
    hd = dirs[0]["w_hh"].shape[1]
    x = g.leaf(x_arr)
    h0l = g.leaf(np.zeros(hd, np.float32) if h0 is None else h0)
    c0l = g.leaf(np.zeros(hd, np.float32) if c0 is None else c0)
    out, _, _ = lstm_run(g, x, h0l, c0l, dirs[0], False, wtype)
    if len(dirs) == 1:
        return out
    rout, _, _ = lstm_run(g, x, h0l, c0l, dirs[1], True, wtype)
    T = x_arr.shape[0]
    return g.node("CONCAT", F32, [2 * hd, T], [out, rout], params=[0])


def ref_lstm(x, dirs, h0=None, c0=None):
    """float64 torch.nn.LSTM (batch 1, one layer): x (T, in) -> (T, H * n_dirs)."""
    def sig(v):
        return 1.0 / (1.0 + np.exp(-v))
    outs = []
    for di, d in enumerate(dirs):
        hd = d["w_hh"].shape[1]
        h = np.zeros(hd) if h0 is None else h0.astype(np.float64)
        c = np.zeros(hd) if c0 is None else c0.astype(np.float64)
        ys = np.zeros((x.shape[0], hd))
        order = range(x.shape[0]) if di == 0 else range(x.shape[0] - 1, -1, -1)
        for t in order:
            z = d["w_ih"].astype(np.float64) @ x[t] + d["b_ih"] + d["w_hh"].astype(np.float64) @ h + d["b_hh"]
            i, f, gg, o = sig(z[:hd]), sig(z[hd:2 * hd]), np.tanh(z[2 * hd:3 * hd]), sig(z[3 * hd:])
            c = f * c + i * gg
            h = o * np.tanh(c)
            ys[t] = h
        outs.append(ys)
    return np.concatenate(outs, 1)
