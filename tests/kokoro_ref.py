"""Float32 PyTorch restatement of Kokoro's iSTFTNet generator (test infrastructure only).

It follows the published Kokoro-82M PyTorch model (istftnet.py: Generator, AdaINResBlock1,
AdaIN1d, SineGen / SourceModuleHnNSF, TorchSTFT) in the form the reference builds it
(/root/reference/src/models/kokoro/model.cpp:136-244):
  - the sine source runs at the frame rate: phases = cumsum(((f0 * (h+1)/sr) mod 1)) * 2*pi*300,
    then linear x300 interpolation (model.cpp:172-176), without SineGen's random initial phase;
  - uv and the noise draws come from the same host arrays the runner uploads
    (uv_noise_compute, util.cpp:140-170: uniform draws, noise_std when voiced else sin_amp / 3);
  - the iSTFT is divided by compute_window_squared_sum's envelope (util.cpp:203-217), which
    matches torch.istft's envelope except for one extra frame at the end (its window tail lands
    on the last hop - 1 samples): callers compare all but the last `hop` samples.
Convolutions here are fp32 (ggml's conv_1d rounds im2col and kernels to f16), so agreement with
the oracle is at the f16 level, not bit level.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def hann(n):
    return torch.tensor([np.float32(math.sin(math.pi * i / n) ** 2) for i in range(n)], dtype=torch.float32)


def _snake(x, alpha):
    a = alpha.reshape(1, -1, 1)
    return x + (1.0 / a) * torch.sin(a * x) ** 2


def _adain(x, style, gw, gb, bw, bb):
    gamma = (gw @ style + gb).reshape(1, -1, 1)
    beta = (bw @ style + bb).reshape(1, -1, 1)
    xn = F.instance_norm(x, eps=1e-5)
    return xn + xn * gamma + beta


def _res_block(W, pre, x, style, kernel, dilations):
    """AdaINResBlock1 (three units; conv2 undilated with padding (k-1)/2)."""
    for i in range(3):
        p = f"{pre}.{i}"
        xt = _adain(x, style, W[p + ".gamma1_weight"], W[p + ".gamma1_bias"], W[p + ".beta1_weight"], W[p + ".beta1_bias"])
        xt = _snake(xt, W[p + ".alpha1"])
        d = dilations[i]
        xt = F.conv1d(xt, W[p + ".convs1_weight"], W[p + ".convs1_bias"].reshape(-1), padding=d * (kernel - 1) // 2, dilation=d)
        xt = _adain(xt, style, W[p + ".gamma2_weight"], W[p + ".gamma2_bias"], W[p + ".beta2_weight"], W[p + ".beta2_bias"])
        xt = _snake(xt, W[p + ".alpha2"])
        xt = F.conv1d(xt, W[p + ".convs2_weight"], W[p + ".convs2_bias"].reshape(-1), padding=(kernel - 1) // 2)
        x = x + xt
    return x


def uv_noise(cfg, f0, rand):
    """uv_noise_compute over the nearest-x300 F0 (host side in both runner and reference)."""
    T = f0.shape[0]
    L = 300 * T
    sf = np.float32(L) / np.float32(T)
    idx = (np.arange(L, dtype=np.float32) / sf).astype(np.int64)
    voiced = f0[idx] > np.float32(cfg.voice_threshold)
    uv = np.where(voiced, np.float32(cfg.sin_amp), np.float32(0)).astype(np.float32)
    amp = np.where(voiced, np.float32(cfg.noise_std), np.float32(cfg.sin_amp) / np.float32(3)).astype(np.float32)
    return np.broadcast_to(uv, rand.shape).astype(np.float32), (amp[None, :] * rand).astype(np.float32)


def _f16(t):
    return t.to(torch.float16).to(torch.float32)


def generator(cfg, W, x, f0, style, rand, taps=None, har_branch=None, f16=False):
    """x: (T, C) features, f0: (T,), style: (S,), rand: (H, 300T) -> (300T,) float32 PCM.
    taps: optional dict filled with the runner's named intermediates in its memory order.
    har_branch: the runner's "har_spec" node; where a phase sits on the +-pi branch cut (a real
    negative bin, e.g. frame 0, which reflect padding makes even) the two atan2s may land on
    opposite sides, so this restatement takes the runner's side of the cut (a 2*pi shift, not
    a substitution of values).
    f16: the F16 model (Kokoro weight_type F16): ggml's F16 mul_mat / conv_transpose_1d round
    their input to f16 (vec_dot_type; conv_transpose_1d_f16_f32), so the sine merge and the
    upsamplers see f16-rounded inputs here too."""
    taps = {} if taps is None else taps
    W = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in W.items()}
    T = x.shape[0]
    H = cfg.harmonic_num + 1
    n_fft, hop = cfg.n_fft, cfg.hop
    nb = n_fft // 2 + 1
    xs = torch.from_numpy(np.ascontiguousarray(x.T))[None]  # [1, C, T]
    s = torch.from_numpy(style)
    f0t = torch.from_numpy(f0)
    hn = torch.tensor([(np.float32(i) + np.float32(1)) / np.float32(cfg.sample_rate) for i in range(H)], dtype=torch.float32)
    rad = torch.fmod(f0t[:, None] * hn[None, :], 1.0)  # [T, H]
    phase = torch.cumsum(rad.double(), 0).float() * torch.tensor(np.float32(600.0 * math.pi))
    up = F.interpolate(phase.T[None], scale_factor=300, mode="linear", align_corners=False)[0]  # [H, 300T]
    uv, noise = uv_noise(cfg, f0, rand)
    sines = torch.sin(up) * torch.from_numpy(uv) + torch.from_numpy(noise)
    taps["sine_source"] = sines.T
    har = torch.tanh(W["gen.m_source_weight"].reshape(1, H) @ (_f16(sines) if f16 else sines) + W["gen.m_source_bias"].reshape(1, 1))
    win = hann(n_fft)
    spec = torch.stft(har, n_fft, hop, n_fft, window=win, center=True, pad_mode="reflect", return_complex=True)  # [1, nb, F]
    # the DFT of a real signal has an exactly real DC / Nyquist bin; torch's FFT leaves +-tiny
    # imaginary noise there, whose sign flips angle() between 0 and +-pi.  The fork's STFT sets the
    # imaginary part to +0 (oracle/ggml_ref.c op_stft), and so does this restatement.
    for b in (0, n_fft // 2) if n_fft % 2 == 0 else (0,):
        spec[:, b, :] = torch.complex(spec[:, b, :].real, torch.zeros_like(spec[:, b, :].real))
    ang = spec.angle()
    if har_branch is not None:
        ref = torch.from_numpy(np.asarray(har_branch, dtype=np.float32).reshape(2 * nb, -1)[nb:])[None]
        ang = torch.where((ang - ref).abs() > math.pi, ang + 2 * math.pi * torch.sign(ref - ang), ang)
    har = torch.cat([spec.abs(), ang], dim=1)
    taps["har_spec"] = har[0]
    for i in range(cfg.n_ups):
        xs = F.leaky_relu(xs, 0.1)
        g = f"gen.ups.{i}"
        k, r = cfg.up_kernels[i], cfg.up_rates[i]
        xs = F.conv_transpose1d(_f16(xs) if f16 else xs, W[g + ".weight"], W[g + ".bias"].reshape(-1), stride=r, padding=(k - r) // 2)
        if i == cfg.n_ups - 1:
            xs = F.pad(xs, (1, 0), mode="reflect")
        taps[f"up.{i}"] = xs[0]
        n = f"gen.noise_blocks.{i}"
        sf0 = int(np.prod([cfg.up_rates[j] for j in range(i + 1, cfg.n_ups)])) if i + 1 < cfg.n_ups else 1
        src = F.conv1d(har, W[n + ".input_conv.weight"], W[n + ".input_conv.bias"].reshape(-1), stride=sf0,
                       padding=(sf0 + 1) // 2 if sf0 > 1 else 0)
        taps[f"noise_conv.{i}"] = src[0]
        src = _res_block(W, n + ".res_block", src, s, cfg.noise_res_kernels[i], list(cfg.res_dilations))
        taps[f"noise_res.{i}"] = src[0]
        xs = xs + src
        acc = None
        for j in range(cfg.n_kernels):
            rb = _res_block(W, f"gen.res_blocks.{i * cfg.n_kernels + j}", xs, s, cfg.res_kernels[j], list(cfg.res_dilations))
            acc = rb if acc is None else acc + rb
        xs = acc / cfg.n_kernels
        taps[f"level.{i}"] = xs[0].T
    xs = F.leaky_relu(xs, 0.01)
    xs = F.conv1d(xs, W["gen.conv_post.weight"], W["gen.conv_post.bias"].reshape(-1), padding=3)
    taps["conv_post"] = xs[0]
    mag = torch.exp(xs[:, :nb, :])
    ph = torch.sin(xs[:, nb:, :])
    pcm = torch.istft(mag * torch.exp(ph * 1j), n_fft, hop, n_fft, window=win, center=True)
    return pcm[0].numpy().astype(np.float32)
