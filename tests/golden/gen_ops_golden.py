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
    np.savez_compressed(OUT, **d)
    print("wrote", OUT, sorted(d))


if __name__ == "__main__":
    main()
