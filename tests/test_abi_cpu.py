"""C-ABI boundary checks that need no GPU: the shared library loads, exports every function
include/*.h declares, the tts_tensor layout ctypes uses equals the C compiler's, and the host-side
entry points (type traits, Q4_K lane repack, supports_op) behave as documented."""
import ctypes
import pathlib
import re
import subprocess

import numpy as np
import pytest

import ttship

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADERS = sorted((ROOT / "include").glob("*.h"))

_DECL = re.compile(r"^[A-Za-z_][\w\s\*]*?\b(tts_\w+)\s*\(", re.M)


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def declared_functions():
    names = set()
    for h in HEADERS:
        body = _strip_comments(h.read_text())
        for m in _DECL.finditer(body):
            line = body[m.start():body.find("\n", m.start())]
            if line.lstrip().startswith(("typedef", "struct", "enum", "#")):
                continue
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_entry_points():
    names = declared_functions()
    for must in ("tts_hip_backend_init", "tts_hip_graph_compute", "tts_hip_supports_op", "tts_hip_tensor_get",
                 "tts_parler_create", "tts_parler_generate", "tts_repack_q4_K"):
        assert must in names
    assert len(names) >= 35


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports(name):
    lib = ctypes.CDLL(str(ttship.LIB_PATH))
    assert hasattr(lib, name), f"{name} declared in include/ but not exported by {ttship.LIB_PATH.name}"


def test_tensor_layout_matches_c(tmp_path):
    """ctypes' TtsTensor / BackendIface must match the C layout field by field."""
    fields = [f for f, _ in ttship.TtsTensor._fields_]
    prog = ["#include <stdio.h>", "#include <stddef.h>", '#include "tts_hip.h"', "int main(void){",
            'printf("%zu\\n", sizeof(tts_tensor));']
    prog += [f'printf("%zu\\n", offsetof(tts_tensor, {f}));' for f in fields]
    prog += ['printf("%zu\\n", sizeof(tts_backend_iface));', "return 0;}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(prog))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert out[0] == ctypes.sizeof(ttship.TtsTensor)
    for f, off in zip(fields, out[1:-1]):
        assert getattr(ttship.TtsTensor, f).offset == off, f
    assert out[-1] == ctypes.sizeof(ttship.BackendIface)


def test_type_traits():
    L = ttship.lib()
    assert (L.tts_type_size(ttship.Q4_K), L.tts_blck_size(ttship.Q4_K)) == (144, 256)
    assert (L.tts_type_size(ttship.Q8_0), L.tts_blck_size(ttship.Q8_0)) == (34, 32)
    assert (L.tts_type_size(ttship.F16), L.tts_type_size(ttship.F32)) == (2, 4)
    assert L.tts_row_size(ttship.Q4_K, 1024) == 4 * 144
    assert L.tts_row_size(ttship.Q8_0, 2048) == 64 * 34
    for i, n in enumerate(ttship.OPS):
        assert L.tts_op_name(i).decode() == n


def test_repack_q4_K_roundtrip_and_layout():
    L = ttship.lib()
    rng = np.random.default_rng(7)
    nb = 37
    src = rng.integers(0, 256, size=nb * 144, dtype=np.uint8)
    rep = np.empty_like(src)
    back = np.empty_like(src)
    L.tts_repack_q4_K(src.ctypes.data, rep.ctypes.data, nb, 0)
    L.tts_repack_q4_K(rep.ctypes.data, back.ctypes.data, nb, 1)
    assert np.array_equal(back, src)
    s = src.reshape(nb, 144)
    r = rep.reshape(nb, 144)
    assert np.array_equal(r[:, :16], s[:, :16])            # d, dmin, scales untouched
    for l in range(8):
        for c in range(4):
            for k in range(4):
                assert np.array_equal(r[:, 16 + l * 16 + c * 4 + k], s[:, 16 + 32 * c + 8 * k + l])


def _t(type_, ne, op=0, srcs=(), flags=0):
    t = ttship.TtsTensor()
    t.type, t.op, t.flags = type_, op, flags
    for i in range(4):
        t.ne[i] = ne[i] if i < len(ne) else 1
    ts = ttship.TYPE_SIZE.get(type_, 4)
    bs = ttship.BLCK_SIZE.get(type_, 1)
    t.nb[0] = ts
    t.nb[1] = ts * (t.ne[0] // bs)
    t.nb[2] = t.nb[1] * t.ne[1]
    t.nb[3] = t.nb[2] * t.ne[2]
    for i, s in enumerate(srcs):
        t.src[i] = ctypes.pointer(s)
    return t


def test_supports_op_host_logic():
    L = ttship.lib()
    L.tts_hip_supports_op.argtypes = [ctypes.POINTER(ttship.TtsTensor)]
    x = _t(ttship.F32, [1024, 1])
    w = _t(ttship.Q4_K, [1024, 1024])
    mm = _t(ttship.F32, [1024, 1], op=ttship.OP["MUL_MAT"], srcs=(w, x))
    assert L.tts_hip_supports_op(ctypes.byref(mm)) == 1
    w_bad = _t(ttship.Q4_K, [1000 // 256 * 256 + 256, 4])
    w_bad.ne[0] = 1000
    mm_bad = _t(ttship.F32, [4, 1], op=ttship.OP["MUL_MAT"], srcs=(w_bad, x))
    assert L.tts_hip_supports_op(ctypes.byref(mm_bad)) == 0
    # ggml_can_mul_mat: src1 must broadcast over src0 (dims 2, 3); H = 24 probabilities x 8 V heads is invalid
    kq = _t(ttship.F32, [300, 1, 24, 1])
    v8 = _t(ttship.F32, [300, 64, 8, 1])
    assert L.tts_hip_supports_op(ctypes.byref(_t(ttship.F32, [1, 64, 24, 1], op=ttship.OP["MUL_MAT"], srcs=(kq, v8)))) == 0
    v24 = _t(ttship.F32, [300, 64, 24, 1])
    assert L.tts_hip_supports_op(ctypes.byref(_t(ttship.F32, [1, 64, 24, 1], op=ttship.OP["MUL_MAT"], srcs=(kq, v24)))) == 1
    # buffer-less host leaf (src/util.cpp:86-94 reciprocal) must stay on the CPU backend
    host_leaf = _t(ttship.F32, [1024, 1], flags=2)
    div = _t(ttship.F32, [1024, 1], op=ttship.OP["DIV"], srcs=(x, host_leaf))
    assert L.tts_hip_supports_op(ctypes.byref(div)) == 0
    add = _t(ttship.F32, [1024, 1], op=ttship.OP["ADD"], srcs=(x, x))
    assert L.tts_hip_supports_op(ctypes.byref(add)) == 1


def test_no_device_is_reported_not_faked():
    """Without a GPU the product path must refuse, not fall back to a CPU implementation."""
    L = ttship.lib()
    if L.tts_hip_device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(RuntimeError):
        ttship.HipBackend(0)


def test_repack_q4_K_tiled_roundtrip_and_layout():
    """4-row tile layout (include/tts_hip.h): per (tile, block) 576 B = 4 headers, then 16-B pieces
    (chunk c, half h, row i) whose dword l' holds qs[32c + 8kk + 4h + l'], kk = 0..3."""
    L = ttship.lib()
    rng = np.random.default_rng(11)
    N, nb = 12, 3
    src = rng.integers(0, 256, size=N * nb * 144, dtype=np.uint8)
    til = np.empty_like(src)
    back = np.empty_like(src)
    L.tts_repack_q4_K_tiled(src.ctypes.data, til.ctypes.data, N, nb, 0)
    L.tts_repack_q4_K_tiled(til.ctypes.data, back.ctypes.data, N, nb, 1)
    assert np.array_equal(back, src)
    s = src.reshape(N, nb, 144)
    t = til.reshape(N // 4, nb, 576)
    for row in range(N):
        for b in range(nb):
            g, i = t[row // 4, b], row % 4
            assert np.array_equal(g[i * 16:i * 16 + 16], s[row, b, :16])
            for c in range(4):
                for h in range(2):
                    piece = g[64 + ((c * 2 + h) * 4 + i) * 16:][:16]
                    for lp in range(4):
                        for kk in range(4):
                            assert piece[lp * 4 + kk] == s[row, b, 16 + 32 * c + 8 * kk + 4 * h + lp]
