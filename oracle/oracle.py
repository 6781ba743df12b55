"""ctypes wrapper of the CPU oracle (oracle/oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker / the reported CPU baseline, never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "oracle.cpp")):
            build()
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        lib.orc_create.restype = P
        lib.orc_create.argtypes = [P, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int]
        lib.orc_destroy.argtypes = [P]
        lib.orc_push.restype = ctypes.c_int
        lib.orc_push.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, P, P, P, P, P, P, ctypes.c_char_p, ctypes.c_int]
        lib.orc_output_count.restype = ctypes.c_int64
        lib.orc_output_count.argtypes = [P]
        lib.orc_fetch.restype = ctypes.c_int64
        lib.orc_fetch.argtypes = [P, ctypes.c_int64, P, P, P, P, P, P]
        lib.orc_advance_time.argtypes = [P, ctypes.c_int64, ctypes.c_uint64]
        _lib = lib
    return _lib


class OracleEngine:
    """Engine-interface implementation backed by the oracle (see siddhi_amd/runtime.py)."""

    def __init__(self, ctx):
        from siddhi_amd import lowering as L
        lib = _load()
        self.ctx = ctx
        self.nsel = len(ctx.query.select)
        img = np.array(L.oracle_image(ctx), dtype=np.int64)
        err = ctypes.create_string_buffer(512)
        self.h = lib.orc_create(img.ctypes.data, len(img), err, 512)
        if not self.h:
            raise RuntimeError("oracle: " + err.value.decode())
        self._keep = img

    def push(self, b):
        lib = _load()
        ncols = len(b.cols)
        cols = (ctypes.c_void_p * ncols)(*[c.ctypes.data for c in b.cols])
        nul = (ctypes.c_void_p * ncols)(*[(x.ctypes.data if x is not None else None) for x in b.nulls])
        err = ctypes.create_string_buffer(512)
        ts = np.ascontiguousarray(b.ts, dtype=np.int64)
        st = np.ascontiguousarray(b.stream, dtype=np.int32)
        ky = np.ascontiguousarray(b.key, dtype=np.int32)
        ix = None
        if getattr(b, "index", None) is not None:
            ixa = np.ascontiguousarray(b.index, np.uint64)
            ix = ixa.ctypes.data
        rc = lib.orc_push(self.h, b.n, b.base_index, ts.ctypes.data, st.ctypes.data, ky.ctypes.data, ix,
                          ctypes.cast(cols, ctypes.c_void_p), ctypes.cast(nul, ctypes.c_void_p), err, 512)
        if rc != 0:
            raise RuntimeError("oracle: " + err.value.decode())

    def fetch(self):
        from siddhi_amd.runtime import Outputs
        lib = _load()
        n = lib.orc_output_count(self.h)
        tr = np.zeros(n, np.uint64)
        ts = np.zeros(n, np.int64)
        ky = np.zeros(n, np.int32)
        gr = np.zeros(n, np.uint32)
        vals = np.zeros((n, self.nsel), np.int64)
        vn = np.zeros((n, self.nsel), np.uint8)
        if n:
            lib.orc_fetch(self.h, n, tr.ctypes.data, ts.ctypes.data, ky.ctypes.data, gr.ctypes.data,
                          vals.ctypes.data, vn.ctypes.data)
        return Outputs(tr, ts, ky, gr, vals, vn)

    def close(self):
        if self.h:
            _load().orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
