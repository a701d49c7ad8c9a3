"""TEST INFRASTRUCTURE ONLY: ctypes loader for the CPU oracle (oracle/ggml_ref.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import pathlib
import subprocess
import sys

_HERE = pathlib.Path(__file__).resolve().parent
LIB = _HERE / "_build" / "liboracle.so"
sys.path.insert(0, str(_HERE.parent / "tts.cpp_amd"))
import ttship  # noqa: E402

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB.exists():
        subprocess.check_call(["make", "-C", str(_HERE)])
    L = ctypes.CDLL(str(LIB))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    sig = {
        "ref_fp16_to_fp32": (ctypes.c_float, [ctypes.c_uint16]),
        "ref_fp32_to_fp16": (ctypes.c_uint16, [ctypes.c_float]),
        "ref_dequantize_row_q4_K": (None, [vp, vp, i64]),
        "ref_dequantize_row_q8_0": (None, [vp, vp, i64]),
        "ref_quantize_row_q8_K": (None, [vp, vp, i64]),
        "ref_quantize_row_q8_0": (None, [vp, vp, i64]),
        "ref_quantize_row_q4_K": (None, [vp, vp, i64]),
        "ref_vec_dot_q4_K_q8_K": (None, [ctypes.c_int, vp, vp, vp]),
        "ref_vec_dot_q8_0_q8_0": (None, [ctypes.c_int, vp, vp, vp]),
        "ref_gelu_f32": (ctypes.c_float, [ctypes.c_float]),
        "ref_gelu_table": (ctypes.c_float, [ctypes.c_float]),
        "ref_gemv": (None, [ctypes.c_int, vp, vp, vp, i64, i64, i64, ctypes.c_int]),
        "oracle_graph_compute": (ctypes.c_int, [ctypes.POINTER(ctypes.POINTER(ttship.TtsTensor)), ctypes.c_int, ctypes.c_int]),
        "oracle_compute_node": (ctypes.c_int, [ctypes.POINTER(ttship.TtsTensor)]),
        "oracle_backend_iface": (ctypes.c_int, [ctypes.POINTER(ttship.BackendIface), ctypes.c_int]),
        "oracle_set_simd_mode": (None, [ctypes.c_int]),
        "oracle_simd_mode": (ctypes.c_int, []),
        "ref_vec_dot_f16": (None, [ctypes.c_int, vp, vp, vp]),
        "ref_vec_dot_f32": (None, [ctypes.c_int, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class simd_mode:
    """with simd_mode(1): the oracle accumulates like an x86 AVX2/FMA/F16C ggml-cpu build (ggml_ref.c)."""

    def __init__(self, mode=1):
        self.mode = mode

    def __enter__(self):
        self.prev = lib().oracle_simd_mode()
        lib().oracle_set_simd_mode(self.mode)
        return self

    def __exit__(self, *a):
        lib().oracle_set_simd_mode(self.prev)


def iface(n_threads=8):
    it = ttship.BackendIface()
    lib().oracle_backend_iface(ctypes.byref(it), n_threads)
    return it


def gemv(wtype, w_bytes, x, N, n_threads=8):
    """y[M][N] = W[N][K] . x[M][K] with ggml-cpu semantics."""
    import numpy as np
    x = np.ascontiguousarray(x, dtype=np.float32)
    M, K = x.shape
    y = np.empty((M, N), dtype=np.float32)
    w = np.ascontiguousarray(w_bytes)
    lib().ref_gemv(wtype, w.ctypes.data, x.ctypes.data, y.ctypes.data, K, N, M, n_threads)
    return y


def dequant_q4_K(w_bytes, K, N):
    import numpy as np
    w = np.ascontiguousarray(w_bytes, dtype=np.uint8).reshape(-1)
    out = np.empty((N, K), dtype=np.float32)
    rs = K // 256 * 144
    for n in range(N):
        lib().ref_dequantize_row_q4_K(w[n * rs:].ctypes.data, out[n].ctypes.data, K)
    return out


def dequant_q8_0(w_bytes, K, N):
    import numpy as np
    w = np.ascontiguousarray(w_bytes, dtype=np.uint8).reshape(-1)
    out = np.empty((N, K), dtype=np.float32)
    rs = K // 32 * 34
    for n in range(N):
        lib().ref_dequantize_row_q8_0(w[n * rs:].ctypes.data, out[n].ctypes.data, K)
    return out


def quantize(wtype, x):
    """quantize_row_q4_K_ref / quantize_row_q8_0_ref over the rows of x [N][K] -> ggml bytes."""
    import numpy as np
    x = np.ascontiguousarray(x, dtype=np.float32)
    N, K = x.shape
    rs = K // 256 * 144 if wtype == ttship.Q4_K else K // 32 * 34
    out = np.zeros(N * rs, dtype=np.uint8)
    fn = lib().ref_quantize_row_q4_K if wtype == ttship.Q4_K else lib().ref_quantize_row_q8_0
    for n in range(N):
        fn(x[n].ctypes.data, out[n * rs:].ctypes.data, K)
    return out
