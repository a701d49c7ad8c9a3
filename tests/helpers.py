"""Shared test helpers: synthetic quant blocks, tolerance checks."""
import numpy as np


def rand_q4_K(rng, N, K):
    """Random valid Q4_K rows (any bit pattern of scales/nibbles is a valid block)."""
    nb = K // 256
    blk = np.zeros((N, nb, 144), dtype=np.uint8)
    d = (rng.uniform(0.5, 1.5, size=(N, nb)) * 1e-3).astype(np.float16)
    dmin = (rng.uniform(0.5, 1.5, size=(N, nb)) * 4e-3).astype(np.float16)
    blk[:, :, 0:2] = d.view(np.uint8).reshape(N, nb, 2)
    blk[:, :, 2:4] = dmin.view(np.uint8).reshape(N, nb, 2)
    blk[:, :, 4:] = rng.integers(0, 256, size=(N, nb, 140), dtype=np.uint8)
    return blk.reshape(N, nb * 144)


def rand_q8_0(rng, N, K):
    nb = K // 32
    blk = np.zeros((N, nb, 34), dtype=np.uint8)
    d = (rng.uniform(0.5, 1.5, size=(N, nb)) * 2e-3).astype(np.float16)
    blk[:, :, 0:2] = d.view(np.uint8).reshape(N, nb, 2)
    q = rng.integers(-127, 128, size=(N, nb, 32)).astype(np.int8)
    blk[:, :, 2:] = q.view(np.uint8)
    return blk.reshape(N, nb * 34)


def assert_close_scaled(got, ref, scale, rtol, what=""):
    """|got-ref| <= rtol * scale elementwise (scale = sum |w||x| style magnitude)."""
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    bound = rtol * np.maximum(scale, 1e-30)
    bad = err > bound
    if bad.any():
        i = np.argmax(err / bound)
        raise AssertionError(f"{what}: {bad.sum()} / {err.size} exceed tol; worst idx {i} got {got.flat[i]} ref {ref.flat[i]} "
                             f"err {err.flat[i]:.3e} bound {bound.flat[i]:.3e}")
