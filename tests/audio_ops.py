"""Node builders for the fork's audio ops (Kokoro sine source and iSTFTNet head),
shared by the oracle-vs-torch and HIP-vs-oracle tests.  Shapes follow ggml's ne order:
  CUMSUM   a [T, R]            -> [T, R]                (cumsum along ne0, build_sin_gen model.cpp:175)
  UPSCALE  a [T, R]            -> [T*s, R]   mode 0 nearest (ggml_upscale_ext), 1 linear (fork)
  STFT     x [L, B], win [N]   -> [N, L/hop+1, B, 2]    (ggml_stft, src/util.cpp:111-120)
  ISTFT    z [N/2+1, F, B, 2], win [N] -> [(F-1)*hop, B] (ggml_istft, src/util.cpp:122-130)"""
import numpy as np

import ttship

F32 = ttship.F32


def cumsum(g, x):
    xl = g.leaf(x) if isinstance(x, np.ndarray) else x
    return g.node("CUMSUM", F32, [xl.ne[i] for i in range(4)], [xl])


def upscale(g, x, ne0, mode):
    xl = g.leaf(x) if isinstance(x, np.ndarray) else x
    return g.node("UPSCALE", F32, [ne0] + [xl.ne[i] for i in range(1, 4)], [xl], params=[mode])


def stft(g, x, win, n_fft, hop, abs_angle=1):
    """x: (B, L) samples."""
    xl = g.leaf(x) if isinstance(x, np.ndarray) else x
    L, B = xl.ne[0], xl.ne[1]
    F = (L + 2 * (n_fft // 2) - n_fft) // hop + 1
    return g.node("STFT", F32, [n_fft, F, B, 2], [xl, g.leaf(win)], params=[n_fft, hop, abs_angle])


def istft(g, z, win, n_fft, hop, abs_angle=1):
    """z: (2, B, F, N/2+1) = magnitude/phase (or re/im) planes."""
    zl = g.leaf(z) if isinstance(z, np.ndarray) else z
    F, B = zl.ne[1], zl.ne[2]
    return g.node("ISTFT", F32, [(F - 1) * hop, B], [zl, g.leaf(win)], params=[n_fft, hop, abs_angle])


def window_envelope(win, hop, F):
    """torch.istft's window envelope (sum of win^2 over the overlapping frames, centre-trimmed)."""
    N = len(win)
    env = np.zeros(N + hop * (F - 1), dtype=np.float64)
    for t in range(F):
        env[t * hop:t * hop + N] += win.astype(np.float64) ** 2
    return env[N // 2: N // 2 + hop * (F - 1)].astype(np.float32)


def ulp_diff(a, b):
    """Largest distance in float32 units-in-the-last-place between two arrays of the same shape."""
    ai = np.ascontiguousarray(a, dtype=np.float32).view(np.int32).astype(np.int64)
    bi = np.ascontiguousarray(b, dtype=np.float32).view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return int(np.max(np.abs(ai - bi))) if ai.size else 0
