"""Generates tests/golden/ops_golden.npz with torch 2.10 on CPU (this container only).

The reference tree holds no golden vectors for any op, so these torch-CPU fixtures
pin the oracle's float semantics: each case stores seeded inputs and torch's output.  Fork-op
fixtures (conv_transpose_1d, stft/istft, upscale, cumsum, mod) follow PyTorch semantics, which is
what the fork's ops restate.

Run: python tests/golden/gen_ops_golden.py
"""
import pathlib

import numpy as np
import torch

OUT = pathlib.Path(__file__).resolve().parent / "ops_golden.npz"


def main():
    g = torch.Generator().manual_seed(0x5EED)
    d = {}

    def rn(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale).float()

    # LayerNorm core (ggml_norm, eps 1e-5), rows of 1024
    x = rn(5, 1024, scale=2.0) + 0.5
    d["norm_x"] = x.numpy()
    d["norm_y"] = torch.nn.functional.layer_norm(x.double(), (1024,), eps=1e-5).float().numpy()
    # RMSNorm (ggml_rms_norm, eps 1e-5)
    x = rn(3, 2048)
    d["rms_x"] = x.numpy()
    d["rms_y"] = (x.double() / torch.sqrt((x.double() ** 2).mean(-1, keepdim=True) + 1e-5)).float().numpy()
    # softmax(scale*x + mask) over rows of 77, mask causal-ish
    x = rn(16, 4, 77)
    m = torch.zeros(4, 77)
    m[1, 50:] = -float("inf")
    m[2, :3] = -float("inf")
    d["sm_x"] = x.numpy()
    d["sm_mask"] = m.numpy()
    d["sm_y"] = torch.softmax(x.double() * 0.125 + m.double(), dim=-1).float().numpy()
    # GELU tanh approximation (ggml_gelu)
    x = torch.linspace(-12, 12, 4001).float()
    d["gelu_x"] = x.numpy()
    d["gelu_y"] = torch.nn.functional.gelu(x.double(), approximate="tanh").float().numpy()
    # SiLU
    d["silu_y"] = torch.nn.functional.silu(x.double()).float().numpy()
    # matmul: ggml_mul_mat(a [K,N], b [K,M]) = b @ a^T  -> [M, N]
    a = rn(24, 64)
    b = rn(5, 64)
    d["mm_a"] = a.numpy()
    d["mm_b"] = b.numpy()
    d["mm_y"] = (b.double() @ a.double().T).float().numpy()
    # RoPE NEOX (rotate halves), theta base 500000, freq factors, head dim 128, positions
    hd, nh, T = 128, 3, 4
    x = rn(T, nh, hd)
    pos = torch.tensor([0, 5, 17, 400], dtype=torch.int32)
    ff = torch.linspace(1.0, 8.0, hd // 2).float()
    inv = 500000.0 ** (-torch.arange(0, hd, 2, dtype=torch.float64) / hd) / ff.double()
    ang = pos.double()[:, None] * inv[None, :]
    c, s = torch.cos(ang)[:, None, :], torch.sin(ang)[:, None, :]
    x1, x2 = x.double()[..., : hd // 2], x.double()[..., hd // 2:]
    d["rope_x"] = x.numpy()
    d["rope_pos"] = pos.numpy()
    d["rope_ff"] = ff.numpy()
    d["rope_y"] = torch.cat([x1 * c - x2 * s, x1 * s + x2 * c], -1).float().numpy()
    # conv_transpose_1d (fork op, PyTorch ConvTranspose1d semantics): DAC-style upsampler
    # (K = 2s, p = ceil(s/2), op = s % 2), a depthwise Kokoro-style one, and a dilated one.
    # torch weight layout (IC, OC/g, K) = ggml ne [K, OC/g, IC].
    for name, (IC, OC, L, K, s, p, dil, op, grp) in {
        "ct_dac": (8, 4, 5, 16, 8, 4, 1, 0, 1),
        "ct_dw": (6, 6, 7, 3, 2, 1, 1, 1, 6),
        "ct_dil": (5, 3, 4, 3, 3, 2, 2, 1, 1),
    }.items():
        x = rn(1, IC, L)
        w = rn(IC, OC // grp, K, scale=0.3)
        y = torch.nn.functional.conv_transpose1d(x.double(), w.double(), stride=s, padding=p, output_padding=op,
                                                 groups=grp, dilation=dil)
        d[name + "_x"] = x[0].numpy()
        d[name + "_w"] = w.numpy()
        d[name + "_y"] = y[0].float().numpy()
        d[name + "_prm"] = np.array([s, p, dil, op, grp], dtype=np.int32)
    # conv_1d = im2col(F16) . mul_mat: both operands rounded to fp16, products exact, f64 sums
    IC, OC, L, K, s, p, dil = 16, 12, 40, 7, 1, 9, 3
    x = rn(1, IC, L)
    w = rn(OC, IC, K, scale=0.2)
    y = torch.nn.functional.conv1d(x.half().double(), w.half().double(), stride=s, padding=p, dilation=dil)
    d["c1_x"] = x[0].numpy()
    d["c1_w"] = w.numpy()
    d["c1_y"] = y[0].float().numpy()
    d["c1_prm"] = np.array([s, p, dil], dtype=np.int32)

    # ---- Kokoro sine source / iSTFTNet head (fork ops, float32 torch as Kokoro runs it) ----
    # sine source front: mod 1 -> cumsum (dim of time) -> x600pi -> linear x300
    f0 = torch.rand(1, 23, generator=g) * 400.0
    h = (torch.arange(1, 10).float() / 24000.0)[:, None]
    rad = torch.fmod(f0 * h, 1.0)                         # [9, 23]
    d["sg_f0"] = f0[0].numpy()
    d["sg_rad"] = rad.numpy()
    d["sg_cumsum"] = torch.cumsum(rad, dim=1).numpy()     # CPU: double accumulator
    ph = torch.cumsum(rad, dim=1) * np.float32(600.0 * np.pi)
    d["sg_phase"] = ph.numpy()
    d["sg_up"] = torch.nn.functional.interpolate(ph[None], scale_factor=300, mode="linear")[0].numpy()
    d["sg_f0_up"] = torch.nn.functional.interpolate(f0[None], scale_factor=300, mode="nearest")[0].numpy()
    # linear upscale of a non-integer-friendly length and a 2x factor
    x = rn(3, 7)
    d["ul_x"] = x.numpy()
    d["ul_y2"] = torch.nn.functional.interpolate(x[None], scale_factor=2, mode="linear")[0].numpy()
    d["ul_y5"] = torch.nn.functional.interpolate(x[None], scale_factor=5, mode="linear")[0].numpy()
    # STFT: Kokoro n_fft 20 / hop 5, periodic hann computed as src/util.cpp:132-137 does (float of
    # the double sin^2), center=True reflect, abs & angle; plus a re/im case (n_fft 16, hop 4)
    for name, (N, H, L) in {"stft20": (20, 5, 300 * 4), "stft16": (16, 4, 160)}.items():
        win = torch.tensor([np.float32(np.sin(np.pi * i / N) ** 2) for i in range(N)], dtype=torch.float32)
        x = rn(1, L, scale=0.3)
        S = torch.stft(x, N, H, N, window=win, center=True, pad_mode="reflect", return_complex=True, onesided=False)
        d[name + "_x"] = x[0].numpy()
        d[name + "_win"] = win.numpy()
        d[name + "_abs"] = S.abs()[0].numpy()        # [N, F]
        d[name + "_angle"] = S.angle()[0].numpy()
        d[name + "_re"] = S.real[0].numpy()
        d[name + "_im"] = S.imag[0].numpy()
    # iSTFT of exp(spec) * e^{i sin(phase)} (build_generator), n_fft 20 / hop 5, F frames
    N, H, F = 20, 5, 97
    win = torch.tensor([np.float32(np.sin(np.pi * i / N) ** 2) for i in range(N)], dtype=torch.float32)
    mag = torch.exp(rn(N // 2 + 1, F, scale=0.5))
    pha = torch.sin(rn(N // 2 + 1, F, scale=2.0))
    y = torch.istft((mag * torch.exp(pha * 1j))[None], N, H, N, window=win, center=True)
    d["istft_mag"] = mag.numpy()
    d["istft_phase"] = pha.numpy()
    d["istft_win"] = win.numpy()
    d["istft_y"] = y[0].numpy()                      # [(F-1)*H]
    np.savez_compressed(OUT, **d)
    print("wrote", OUT, sorted(d))


if __name__ == "__main__":
    main()
