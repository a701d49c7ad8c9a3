"""Float PyTorch restatement of Kokoro-82M's front half (test infrastructure only).

It follows the published Kokoro model (kokoro/modules.py: CustomAlbert / AlbertModel, TextEncoder,
ProsodyPredictor with DurationEncoder + AdaLayerNorm, AdainResBlk1d with its depthwise
ConvTranspose1d pool and nearest x2 shortcut; istftnet.py Decoder) in the form TTS.cpp builds it
(/root/reference/src/models/kokoro/model.cpp:938-1047 duration graph, :1141-1242 main graph):
  - ALBERT with static token type 0, post-LayerNorms (eps 1e-12), tanh-GELU, zero attention mask;
  - the DurationEncoder's three LSTM -> AdaLayerNorm (x + x * gamma + beta) -> style concat layers,
    the duration LSTM, sigmoid projection, sum, round, clamp(1, max_dur);
  - the [total, n] duration mask built as kokoro_runner::set_inputs builds it (model.cpp:1263-1275);
  - the F0 / N stacks, text encoder, decoder blocks, then tests/kokoro_ref.py's generator.
LSTMs are float64 (tests/lstm.py ref_lstm).  Convolutions and GEMMs here are fp32 where ggml rounds
conv inputs / kernels to f16 and GELU through its f16 table, so agreement with the oracle is at the
f16 level, not bit level.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from lstm import ref_lstm


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


def _dirs(W, pre):
    """prepare_lstm_tensor's split back into torch.nn.LSTM per-direction blocks."""
    dirs = []
    for part in (".0.", ".0.reverse_"):
        w = [W[f"{pre}{part}weights.{i}"] for i in range(8)]
        b = [W[f"{pre}{part}biases.{i}"].reshape(-1) for i in range(8)]
        dirs.append({"w_ih": np.concatenate(w[0::2], 0), "w_hh": np.concatenate(w[1::2], 0),
                     "b_ih": np.concatenate(b[0::2], 0), "b_hh": np.concatenate(b[1::2], 0)})
    return dirs


def _lstm(W, pre, x):
    """x (T, in) torch -> (T, 2H) torch (float64 recurrence)."""
    return torch.from_numpy(ref_lstm(x.double().numpy(), _dirs(W, pre)).astype(np.float32))


def _ln(x, w=None, b=None, eps=1e-5):
    y = F.layer_norm(x, (x.shape[-1],), eps=eps)
    return y if w is None else y * w + b


def styles(W, n):
    """voice row n - 3: (decoder / generator style, prosody style)."""
    v = W["voice_tensors.synthetic"]
    row = v[n - 3]
    S = row.shape[0] // 2
    return _t(row[:S]), _t(row[S:])


def albert(cfg, W, tokens):
    """tokens (n,) -> (n, hidden)."""
    Wt = {k: _t(v) for k, v in W.items() if k.startswith("albert.")}
    n = len(tokens)
    idx = torch.from_numpy(np.asarray(tokens, np.int64))
    x = Wt["albert.token_embd"][idx] + Wt["albert.position_embd"][torch.arange(n)] + Wt["albert.token_type_embd"]
    x = _ln(x, Wt["albert.norm"], Wt["albert.norm_bias"], 1e-12)
    h = x @ Wt["albert.embd"].T + Wt["albert.embd_bias"]
    hs = cfg.hidden // cfg.n_heads
    for _ in range(cfg.n_recurrence):
        for l in range(cfg.n_layers):
            p = f"albert.layer.{l}"
            q = (h @ Wt[p + ".q"].T + Wt[p + ".q_bias"]).reshape(n, cfg.n_heads, hs).transpose(0, 1)
            k = (h @ Wt[p + ".k"].T + Wt[p + ".k_bias"]).reshape(n, cfg.n_heads, hs).transpose(0, 1)
            v = (h @ Wt[p + ".v"].T + Wt[p + ".v_bias"]).reshape(n, cfg.n_heads, hs).transpose(0, 1)
            a = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(hs), -1) @ v
            a = a.transpose(0, 1).reshape(n, cfg.hidden) @ Wt[p + ".o"].T + Wt[p + ".o_bias"]
            h = _ln(a + h, Wt[p + ".attn_norm"], Wt[p + ".attn_norm_bias"], 1e-12)
            f = F.gelu(h @ Wt[p + ".ffn"].T + Wt[p + ".ffn_bias"], approximate="tanh")
            f = f @ Wt[p + ".ffn_out"].T + Wt[p + ".ffn_out_bias"]
            h = _ln(f + h, Wt[p + ".layer_out_norm"], Wt[p + ".layer_out_norm_bias"], 1e-12)
    return h


def durations(cfg, W, tokens, taps=None):
    """-> (hidden (n, D + S), probs (n, max_dur), lengths (n,)) as the duration graph computes them."""
    taps = {} if taps is None else taps
    dp = "duration_predictor"
    Wt = {k: _t(v) for k, v in W.items() if k.startswith(dp)}
    n = len(tokens)
    _, s = styles(W, n)
    h = albert(cfg, W, tokens)
    taps["albert_out"] = h
    x = h @ Wt[dp + ".encode"].T + Wt[dp + ".encode_bias"]
    x = torch.cat([x, s.expand(n, -1)], -1)
    for l in range(cfg.n_dur_layers):
        x = _lstm(W, f"{dp}.layers.{2 * l}.lstm", x)
        pn = f"{dp}.layers.{2 * l + 1}"
        gamma = Wt[pn + ".gamma_weight"] @ s + Wt[pn + ".gamma_bias"]
        beta = Wt[pn + ".beta_weight"] @ s + Wt[pn + ".beta_bias"]
        x = _ln(x)
        x = x + x * gamma + beta
        x = torch.cat([x, s.expand(n, -1)], -1)
    hidden = x
    taps["duration_hidden_states"] = hidden
    d = _lstm(W, dp + ".duration_lstm", x)
    probs = torch.sigmoid(d @ Wt[dp + ".duration_proj"].T + Wt[dp + ".duration_proj_bias"])
    taps["duration_probs"] = probs
    lengths = torch.clamp(torch.floor(probs.sum(-1) + 0.5), 1, cfg.max_dur)
    return hidden, probs, lengths


def duration_mask(lengths, total):
    """kokoro_runner::set_inputs (model.cpp:1263-1275): row i = frames [running, running + len_i)."""
    n = len(lengths)
    m = np.zeros((n, total), np.float32)
    running = np.float32(0)
    for i in range(n):
        nxt = np.float32(running + np.float32(lengths[i]))
        j = np.arange(total, dtype=np.float32)
        m[i] = ((j >= running) & (j < nxt)).astype(np.float32)
        running = nxt
    return m


def _adain(x, s, gw, gb, bw, bb):
    gamma = (gw @ s + gb).reshape(1, -1, 1)
    beta = (bw @ s + bb).reshape(1, -1, 1)
    xn = F.instance_norm(x, eps=1e-5)
    return xn + xn * gamma + beta


def ada_block(W, pre, x, s):
    """AdainResBlk1d on x (1, C, T)."""
    Wt = lambda k: _t(W[pre + "." + k])  # noqa: E731
    r = _adain(x, s, Wt("norm1_gamma_weight"), Wt("norm1_gamma_bias"), Wt("norm1_beta_weight"), Wt("norm1_beta_bias"))
    r = F.leaky_relu(r, 0.2)
    pool = pre + ".pool_weight" in W
    if pool:
        C = x.shape[1]
        r = F.conv_transpose1d(r, Wt("pool_weight"), Wt("pool_bias").reshape(-1), stride=2, padding=1, output_padding=1, groups=C)
    r = F.conv1d(r, Wt("conv1_weight"), Wt("conv1_bias").reshape(-1), padding=1)
    r = _adain(r, s, Wt("norm2_gamma_weight"), Wt("norm2_gamma_bias"), Wt("norm2_beta_weight"), Wt("norm2_beta_bias"))
    r = F.leaky_relu(r, 0.2)
    r = F.conv1d(r, Wt("conv2_weight"), Wt("conv2_bias").reshape(-1), padding=1)
    sc = x
    if pre + ".conv1x1_weight" in W:
        if pool:
            sc = F.interpolate(sc, scale_factor=2, mode="nearest")
        sc = F.conv1d(sc, Wt("conv1x1_weight")[:, :, None])
    return (r + sc) / math.sqrt(2.0)


def decoder(cfg, W, tokens, hidden, lengths, taps=None):
    """The main graph up to the generator: -> (features (2T, C), f0 (2T,), decoder style).
    hidden (n, D + S), lengths (n,) as the duration graph returned them."""
    taps = {} if taps is None else taps
    dp = "duration_predictor"
    n = len(tokens)
    s2, s = styles(W, n)
    total = int(sum(int(v) for v in lengths))
    mask = _t(duration_mask(lengths, total))  # (n, total)
    en = mask.T @ _t(hidden)  # (total, D + S)
    x = _lstm(W, dp + ".shared_lstm", en)  # (total, D)
    taps["shared_lstm"] = x
    f0 = x.T[None]
    for i in range(3):
        f0 = ada_block(W, f"{dp}.f0_blocks.{i}", f0, s)
    f0 = (_t(W[dp + ".f0_proj_kernel"]).reshape(1, -1) @ f0[0]).reshape(-1) + _t(W[dp + ".f0_proj_bias"]).reshape(-1)
    taps["f0_out"] = f0
    nn_ = x.T[None]
    for i in range(3):
        nn_ = ada_block(W, f"{dp}.n_blocks.{i}", nn_, s)
    nn_ = (_t(W[dp + ".n_proj_kernel"]).reshape(1, -1) @ nn_[0]).reshape(-1) + _t(W[dp + ".n_proj_bias"]).reshape(-1)
    taps["n_out"] = nn_
    # text encoder
    idx = torch.from_numpy(np.asarray(tokens, np.int64))
    t = _t(W["text_encoder.embedding_weight"])[idx].T[None]  # (1, D, n)
    for l in range(cfg.te_depth):
        p = f"text_encoder.layers.{l}"
        t = F.conv1d(t, _t(W[p + ".weight"]), _t(W[p + ".bias"]).reshape(-1), padding=cfg.te_kernel // 2)
        t = _ln(t[0].T, _t(W[p + ".gamma"]), _t(W[p + ".beta"])).T[None]
        t = F.leaky_relu(t, 0.2)
    t = _lstm(W, "text_encoder.lstm", t[0].T)  # (n, D)
    taps["text_encoder"] = t
    asr = t.T @ mask  # (D, total)
    taps["asr"] = asr.T
    # decoder
    f0d = F.conv1d(f0.reshape(1, 1, -1), _t(W["decoder.f0_conv_weight"]).reshape(1, 1, 3), _t(W["decoder.f0_conv_bias"]).reshape(-1),
                   stride=2, padding=1)
    nd = F.conv1d(nn_.reshape(1, 1, -1), _t(W["decoder.n_conv_weight"]).reshape(1, 1, 3), _t(W["decoder.n_conv_bias"]).reshape(-1),
                  stride=2, padding=1)
    xd = torch.cat([asr[None], f0d, nd], 1)
    xd = ada_block(W, "decoder.encoder_block", xd, s2)
    taps["encoder_block"] = xd[0]
    asr_res = F.conv1d(asr[None], _t(W["decoder.asr_conv_weight"])[:, :, None], _t(W["decoder.asr_conv_bias"]).reshape(-1))
    for i in range(cfg.n_decode):
        xd = torch.cat([xd, asr_res, f0d, nd], 1)
        xd = ada_block(W, f"decoder.decoder_blocks.{i}", xd, s2)
        taps[f"decoder_block.{i}"] = xd[0]
    taps["decoder_out"] = xd[0].T
    return xd[0].T.contiguous(), f0, s2
