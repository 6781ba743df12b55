"""TEST-ONLY engine running the GPU kernel's per-key machine (siddhi_amd/csrc/interp.h) on the CPU via
tests/host_interp/harness.cpp, to check the general NFA logic against the oracle without a GPU."""
import ctypes as ct
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "_build", "libhostinterp.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        srcs = [os.path.join(HERE, "harness.cpp"), os.path.join(ROOT, "siddhi_amd", "csrc", "interp.h"),
                os.path.join(ROOT, "siddhi_amd", "csrc", "sg_device.h"), os.path.join(ROOT, "siddhi_amd", "csrc", "chain.h"),
                os.path.join(ROOT, "siddhi_amd", "csrc", "seq.h")]
        stale = lambda: not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(s) for s in srcs)  # noqa
        if stale():
            import fcntl
            os.makedirs(os.path.dirname(LIB), exist_ok=True)
            with open(LIB + ".lock", "w") as lk:   # parallel test workers: one builds, the others wait for it
                fcntl.flock(lk, fcntl.LOCK_EX)
                if stale():
                    tmp = f"{LIB}.{os.getpid()}.tmp"
                    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", tmp, srcs[0]], check=True)
                    os.replace(tmp, LIB)
        lib = ct.CDLL(LIB)
        P = ct.c_void_p
        lib.hi_open.restype = P
        lib.hi_open.argtypes = [P, ct.c_int, ct.c_int, ct.c_int, ct.c_int]
        lib.hi_close.argtypes = [P]
        lib.hi_push.restype = ct.c_int
        lib.hi_push.argtypes = [P, P]
        lib.hi_count.restype = ct.c_int64
        lib.hi_count.argtypes = [P]
        lib.hi_fetch.argtypes = [P, P, P, P, P, P, P]
        lib.hi_set_chunk.argtypes = [P, ct.c_int]
        lib.hi_set_pp.argtypes = [P, ct.c_int]
        lib.hi_pp_rule.restype = ct.c_int
        lib.hi_pp_rule.argtypes = [P]
        lib.hi_pp_shape_c3.restype = ct.c_int
        lib.hi_pp_shape_c3.argtypes = [P]
        lib.hi_sq_shape_c3b.restype = ct.c_int
        lib.hi_sq_shape_c3b.argtypes = [P]
        lib.hi_seq_rule.restype = ct.c_int
        lib.hi_seq_rule.argtypes = [P]
        lib.hi_terms_fast.restype = ct.c_int
        lib.hi_terms_fast.argtypes = [P, ct.c_int]
        lib.hi_set_spec.argtypes = [P, ct.c_int64, ct.c_int64]
        lib.hi_spec_reruns.restype = ct.c_int64
        lib.hi_spec_reruns.argtypes = [P]
        lib.hi_pp_skipped.restype = ct.c_int64
        lib.hi_pp_skipped.argtypes = [P]
        lib.hi_pp_steps.restype = ct.c_int64
        lib.hi_pp_steps.argtypes = [P, P]
        _lib = lib
    return _lib


class HostInterpEngine:
    def __init__(self, ctx, pool=256, chunk_rows=0, pp=True, spec=(0, 0)):
        from siddhi_amd import lowering as L
        from siddhi_amd import _native as N
        self.lib = _load()
        self.N = N
        self.nfa = L.lower(ctx)
        self.desc = N.build_desc(self.nfa)
        self.nsel = len(self.nfa.select)
        self.h = self.lib.hi_open(ct.byref(self.desc), pool, pool, pool, pool)
        self.lib.hi_set_chunk(self.h, chunk_rows)
        self.lib.hi_set_pp(self.h, 1 if pp else 0)   # partial lanes (chain.h) where sg_pp_rule allows, as the GPU
        self.lib.hi_set_spec(self.h, spec[0], spec[1])   # sequence lanes: speculative units of spec[0] rows, spec[1] warm-up

    def push(self, b):
        keep = []
        ts = np.ascontiguousarray(b.ts, np.int64)
        st = np.ascontiguousarray(b.stream, np.int32)
        ky = np.ascontiguousarray(b.key, np.int32)
        cols = [np.ascontiguousarray(c) for c in b.cols]
        keep += [ts, st, ky] + cols
        ix = 0
        if getattr(b, "index", None) is not None:
            ixa = np.ascontiguousarray(b.index, np.uint64)
            keep.append(ixa)
            ix = ixa.ctypes.data
        sb = self.N.make_batch(b.n, b.base_index, ts.ctypes.data, st.ctypes.data, ky.ctypes.data,
                               [c.ctypes.data for c in cols],
                               [(x.ctypes.data if x is not None else 0) for x in b.nulls], 0, 0, keep, index=ix)
        rc = self.lib.hi_push(self.h, ct.byref(sb))
        if rc != 0:
            raise RuntimeError(f"host interp error {rc}")

    def fetch(self):
        from siddhi_amd.runtime import Outputs
        n = self.lib.hi_count(self.h)
        tr = np.zeros(n, np.uint64)
        ts = np.zeros(n, np.int64)
        ky = np.zeros(n, np.int32)
        gr = np.zeros(n, np.uint32)
        vals = np.zeros((n, max(self.nsel, 1)), np.int64)
        vn = np.zeros(n, np.uint32)
        self.lib.hi_fetch(self.h, tr.ctypes.data, ts.ctypes.data, ky.ctypes.data, gr.ctypes.data, vals.ctypes.data,
                          vn.ctypes.data)
        vnull = np.zeros((n, self.nsel), np.uint8)
        for k in range(self.nsel):
            vnull[:, k] = (vn >> np.uint32(k)) & np.uint32(1)
        return Outputs(tr, ts, ky, gr, vals[:, :self.nsel], vnull)

    def reruns(self):
        return self.lib.hi_spec_reruns(self.h)

    def pp_counts(self):
        """partial lanes: (rows stepped, rows skipped by wait terms, lanes started)"""
        lanes = ct.c_int64(0)
        steps = self.lib.hi_pp_steps(self.h, ct.byref(lanes))
        return steps, self.lib.hi_pp_skipped(self.h), lanes.value

    def close(self):
        if self.h:
            self.lib.hi_close(self.h)
            self.h = None
