"""Build tts_tensor graph nodes from Python (ctypes) for op-level parity tests.

A `Graph` owns numpy host arrays; `to_device(hip)` mirrors every leaf to device memory so the same
node list can run on the oracle (host pointers) or the HIP backend (device pointers).
"""
import ctypes

import numpy as np

import ttship

NP = {ttship.F32: np.float32, ttship.F16: np.float16, ttship.I32: np.int32}


def _f2i(v):
    return int(np.array([v], dtype=np.float32).view(np.int32)[0])


class Graph:
    def __init__(self):
        self.tensors = []     # TtsTensor objects (kept alive)
        self.nodes = []
        self.arrays = {}      # id(tensor) -> numpy array (host backing of non-view tensors)
        self.nbytes = {}

    def _new(self, typ, ne, op=0, srcs=(), view_of=None, offs=0, nb=None):
        t = ttship.TtsTensor()
        t.type = typ
        t.op = op
        ne = list(ne) + [1] * (4 - len(ne))
        for i in range(4):
            t.ne[i] = ne[i]
        if nb is None:
            es = ttship.TYPE_SIZE[typ]
            bs = ttship.BLCK_SIZE[typ]
            nb = [es, es * (ne[0] // bs)]
            nb += [nb[1] * ne[1], nb[1] * ne[1] * ne[2]]
        for i in range(4):
            t.nb[i] = nb[i]
        for i, s in enumerate(srcs):
            if s is not None:
                t.src[i] = ctypes.pointer(s)
        t._view_of = view_of
        t._offs = offs
        self.tensors.append(t)
        return t

    def leaf(self, arr=None, typ=ttship.F32, ne=None, raw=None):
        """Leaf from a numpy array (shape reversed to ggml ne) or raw bytes with explicit ne."""
        if raw is not None:
            t = self._new(typ, ne)
            buf = np.ascontiguousarray(raw).view(np.uint8).copy()
        else:
            arr = np.ascontiguousarray(arr, dtype=NP[typ])
            t = self._new(typ, list(arr.shape[::-1]))
            buf = arr.view(np.uint8).reshape(-1).copy()
        self.arrays[id(t)] = buf
        t.data = buf.ctypes.data
        return t

    def node(self, op, typ, ne, srcs, params=(), fparams=None, nb=None):
        t = self._new(typ, ne, op=ttship.OP[op] if isinstance(op, str) else op, srcs=srcs, nb=nb)
        for i, p in enumerate(params):
            t.op_params[i] = p
        if fparams:
            for i, v in fparams.items():
                t.op_params[i] = _f2i(v)
        n = int(np.prod(ne)) * ttship.TYPE_SIZE[typ] // ttship.BLCK_SIZE[typ] if nb is None else None
        buf = np.zeros(max(n or 0, 1) + 256, dtype=np.uint8)
        self.arrays[id(t)] = buf
        t.data = buf.ctypes.data
        self.nodes.append(t)
        return t

    def view(self, a, ne, nb, offs=0, op="VIEW"):
        t = self._new(a.type, ne, op=ttship.OP[op], srcs=(a,), view_of=a, offs=offs, nb=nb)
        base = a
        while getattr(base, "_view_of", None) is not None:
            offs += base._offs
            base = base._view_of
        t._root = base
        t._root_offs = offs
        t.data = base.data + offs
        self.nodes.append(t)
        return t

    def permute(self, a, ax):
        ne = [0] * 4
        nb = [0] * 4
        for i in range(4):
            ne[ax[i]] = a.ne[i]
            nb[ax[i]] = a.nb[i]
        t = self.view(a, ne, nb, 0, op="PERMUTE")
        for i in range(4):
            t.op_params[i] = ax[i]  # ggml_permute's op params (the attention fusion matches on them)
        return t

    def transpose(self, a):
        return self.permute(a, (1, 0, 2, 3))

    def node_array(self, t, shape=None, dtype=np.float32):
        buf = self.arrays[id(t)]
        n = int(np.prod([t.ne[i] for i in range(4)]))
        out = buf[: n * np.dtype(dtype).itemsize].view(dtype).copy()
        return out.reshape(shape if shape is not None else [t.ne[i] for i in range(3, -1, -1)])

    def node_ptrs(self):
        arr = (ctypes.POINTER(ttship.TtsTensor) * len(self.nodes))()
        for i, n in enumerate(self.nodes):
            arr[i] = ctypes.pointer(n)
        return arr

    # ---- execution ----
    def run_oracle(self, n_threads=4):
        import py_oracle
        st = py_oracle.lib().oracle_graph_compute(self.node_ptrs(), len(self.nodes), n_threads)
        assert st == 0, st

    def run_hip(self, hip):
        """Copy every backing array to device, point tensors at device memory, run, copy back."""
        dev = {}
        for t in self.tensors:
            if id(t) in self.arrays:
                buf = self.arrays[id(t)]
                d = hip.alloc(buf.nbytes)
                hip.set(d, buf)
                dev[id(t)] = d
        host = {}
        for t in self.tensors:
            host[id(t)] = t.data
            if id(t) in dev:
                t.data = dev[id(t)]
        for t in self.tensors:
            if getattr(t, "_root", None) is not None:
                t.data = dev[id(t._root)] + t._root_offs
        st = ttship.lib().tts_hip_graph_compute(hip.ptr, self.node_ptrs(), len(self.nodes))
        assert st == 0, st
        hip.sync()
        for t in self.tensors:
            if id(t) in dev:
                hip.get(self.arrays[id(t)], dev[id(t)])
                hip.free(dev[id(t)])
            t.data = host[id(t)]
