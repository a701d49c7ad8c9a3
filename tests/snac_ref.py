"""Float32 PyTorch restatement of the SNAC decoder as Orpheus uses it (test infrastructure only).

It follows the published SNAC model (hubertsiuzdak/snac: snac.py SNAC.decode, layers.py Decoder /
DecoderBlock / NoiseBlock / ResidualUnit / Snake1d; vq.py ResidualVectorQuantize.from_codes) in
the form the reference builds it (/root/reference/src/decoder/snac_model.cpp:86-159,
general_neural_audio_codec.cpp:133-172):
  - each head's codes -> codebook rows -> 1x1 out_proj (+ bias) -> repeat_interleave(stride);
  - depthwise 7-tap input conv, 1x1 up conv, then per block: snake, ConvTranspose1d(k = 2s, s,
    p = ceil(s/2)), + bias, NoiseBlock (x + noise * conv1x1(x), no bias), three residual units
    with depthwise 7-tap dilated convs (dilation 1, 3, 9; padding 3*dilation);
  - snake, 7-tap conv to one channel, tanh.
Snake uses 1/alpha as the reference's snake_1d does (SNAC adds 1e-9 to alpha).  The noise draws
come from the same host array the runner uploads.  Convolutions are fp32 here (ggml's conv_1d
rounds im2col and kernels to f16), so agreement with the oracle is at the f16 level."""
import math

import numpy as np
import torch
import torch.nn.functional as F


def _snake(x, alpha, exact_sin=False):
    a = alpha.reshape(1, -1, 1)
    ax = a * x
    s = torch.sin(ax.double()).float() if exact_sin else torch.sin(ax)  # the oracle's sinf is correctly rounded
    return x + (1.0 / a) * s ** 2


def _b(W, name):
    return W[name].reshape(-1)


def decode(cfg, weights, heads, noise, f16=False, taps=None):
    """f16=True restates the oracle's arithmetic up to summation order: every conv_1d input and
    kernel rounded to f16 as ggml's conv_1d / conv_1d_dw do (im2col F16, vec_dot_type F16), f64
    accumulation of the exact products, conv_transpose_1d in f64, bias added in f32 afterwards, and
    snake's sin correctly rounded (the oracle's ref_sinf)."""
    W = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in weights.items()}
    rnd = (lambda t: t.half().double()) if f16 else (lambda t: t)
    snake = lambda x, a: _snake(x, a, exact_sin=f16)  # noqa: E731

    def conv1d(x, w, b=None, **kw):
        y = F.conv1d(rnd(x), rnd(w), None, **kw)
        y = y.float() if f16 else y
        return y if b is None else y + b.reshape(1, -1, 1)
    T = len(heads[-1])
    x = None
    for i in range(cfg.n_heads):
        cb = W[f"quantizers.{i}.codebook.weight"]  # [codebook_size, codebook_dim]
        z = cb[torch.as_tensor(np.asarray(heads[i], dtype=np.int64))].T[None]  # [1, dim, T_i]
        z = conv1d(z, W[f"quantizers.{i}.out_proj.weight"], _b(W, f"quantizers.{i}.out_proj.bias"))
        z = z.repeat_interleave(cfg.repeats[i], dim=-1)
        x = z if x is None else x + z
    tap = (lambda k, v: taps.__setitem__(k, v[0].contiguous())) if taps is not None else (lambda k, v: None)
    tap("embd", x)
    C = cfg.latent_dim
    x = conv1d(x, W["in.weight"], _b(W, "in.bias"), padding=3, groups=C)
    tap("in_conv", x)
    x = conv1d(x, W["up.weight"], _b(W, "up.bias"))
    tap("up", x)
    nz = torch.from_numpy(np.asarray(noise, dtype=np.float32))
    off, up = 0, 1
    for l in range(cfg.n_layers):
        s = cfg.rates[l]
        up *= s
        p = f"layers.{l}"
        x = snake(x, W[p + ".alpha"])
        if f16:  # the fork's conv_transpose_1d: f32 operands, exact f64 products and sums, one rounding
            x = F.conv_transpose1d(x.double(), W[p + ".weight"].double(), None, stride=s, padding=math.ceil(s / 2)).float()
            x = x + _b(W, p + ".bias").reshape(1, -1, 1)
        else:
            x = F.conv_transpose1d(x, W[p + ".weight"], _b(W, p + ".bias"), stride=s, padding=math.ceil(s / 2))
        tap(f"convt.{l}", x)
        n_l = nz[off:off + up * T]
        off += up * T
        x = x + conv1d(x, W[p + ".noise_weight"]) * n_l.reshape(1, 1, -1)
        tap(f"noise.{l}", x)
        ch = x.shape[1]
        for r in range(3):
            q = f"{p}.residual_unit.{r}"
            d = 3 ** r
            y = snake(x, W[q + ".in_alpha"])
            y = conv1d(y, W[q + ".in_weight"], _b(W, q + ".in_bias"), padding=3 * d, dilation=d, groups=ch)
            y = snake(y, W[q + ".out_alpha"])
            y = conv1d(y, W[q + ".out_weight"], _b(W, q + ".out_bias"))
            x = x + y
            tap(f"ru.{l}.{r}", x)
    x = snake(x, W["alpha_out"])
    x = conv1d(x, W["final.weight"].reshape(1, -1, 7), _b(W, "final.bias"), padding=3)
    return torch.tanh(x).reshape(-1).numpy()
