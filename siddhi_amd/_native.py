"""ctypes binding of libsiddhi_gpu.so (the C-ABI in include/siddhi_gpu.h) and the GpuEngine that
siddhi_amd.runtime drives.  The library is built in-tree (siddhi_amd/csrc/Makefile); there is no CPU
fallback: if the library or a GPU is missing the engine raises."""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

from . import lowering as L

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SIDDHI_GPU_LIB") or os.path.join(HERE, "libsiddhi_gpu.so")   # override: experiments

SG_MAX_STATES, SG_MAX_STREAMS, SG_MAX_SELECT, SG_MAX_RET, SG_MAX_COLS, SG_MAX_CODE = 16, 16, 32, 16, 64, 512
SG_ABI_VERSION = 4

SYMBOLS = ["sg_open", "sg_push", "sg_advance_time", "sg_pending", "sg_poll", "sg_device_records", "sg_discard",
           "sg_flush", "sg_reset", "sg_set_stream", "sg_get_timing", "sg_close", "sg_last_error", "sg_version",
           "sg_snapshot", "sg_restore", "sg_host_alloc", "sg_host_free", "sg_poll_columns", "sg_push_deliver",
           "sg_router_open", "sg_router_route", "sg_router_keys", "sg_router_close", "sg_router_dense_ids",
           "sg_merge_order", "sg_node_open", "sg_node_push", "sg_node_reset", "sg_node_stats_get", "sg_node_keys",
           "sg_node_close", "sg_node_last_error", "sg_node_set_key_dict"]

I32, I64, U64 = ct.c_int32, ct.c_int64, ct.c_uint64


class sg_state_desc(ct.Structure):
    _fields_ = [(n, I32) for n in ("kind", "stream", "is_start", "min_count", "max_count", "logical_type",
                                   "partner", "next_state", "next_every", "within_every", "callback",
                                   "has_selector", "this_last", "prog_off", "prog_len", "local")] + \
               [("waiting_time", I64)]


class sg_receiver_desc(ct.Structure):
    _fields_ = [("stream", I32), ("multi", I32), ("selector", I32), ("n", I32),
                ("pres", I32 * SG_MAX_STATES), ("stab", I32 * SG_MAX_STATES)]


class sg_nfa_desc(ct.Structure):
    _fields_ = [("abi_version", I32), ("type", I32), ("within", I64), ("playback", I32), ("partitioned", I32),
                ("n_states", I32), ("n_streams", I32), ("n_cols", I32), ("n_ret", I32), ("n_select", I32),
                ("n_init", I32), ("n_reset", I32), ("n_update", I32), ("n_start", I32),
                ("states", sg_state_desc * SG_MAX_STATES),
                ("recv_of_stream", I32 * SG_MAX_STREAMS),
                ("receivers", sg_receiver_desc * SG_MAX_STREAMS),
                ("init_order", I32 * SG_MAX_STATES), ("reset_ops", I32 * SG_MAX_STATES),
                ("update_ops", I32 * SG_MAX_STATES), ("start_ids", I32 * SG_MAX_STATES),
                ("col_type", I32 * SG_MAX_COLS), ("col_stream", I32 * SG_MAX_COLS),
                ("ret_col", I32 * SG_MAX_RET), ("ret_type", I32 * SG_MAX_RET),
                ("sel_state", I32 * SG_MAX_SELECT), ("sel_index", I32 * SG_MAX_SELECT),
                ("sel_ret", I32 * SG_MAX_SELECT), ("sel_type", I32 * SG_MAX_SELECT),
                ("shape", I32), ("shape_args", I32 * 8), ("shape_prog_off", I32), ("shape_prog_len", I32),
                ("code_len", I32), ("code", I64 * SG_MAX_CODE),
                ("n_out", I32), ("out_type", I32 * SG_MAX_SELECT), ("out_off", I32 * SG_MAX_SELECT),
                ("out_len", I32 * SG_MAX_SELECT), ("having_off", I32), ("having_len", I32),
                ("n_sched", I32), ("sched_state", I32 * SG_MAX_STATES)]


class sg_options(ct.Structure):
    _fields_ = [("max_batch", I64), ("pool_partials", I32), ("pool_events", I32), ("pool_chain", I32),
                ("list_cap", I32), ("force_general", I32), ("no_carry", I32), ("ring_cap", I32),
                ("chunk_rows", I32), ("walker_only", I32), ("ingress_rows", I32),
                ("partition_sort", I32), ("partial_lanes", I32), ("no_grow", I32), ("bounded_lateness", I32),
                ("max_lateness_ms", I64)]


class sg_batch(ct.Structure):
    _fields_ = [("n", I64), ("base_index", U64), ("ts", ct.c_void_p), ("stream", ct.c_void_p),
                ("key", ct.c_void_p), ("index", ct.c_void_p), ("cols", ct.c_void_p), ("nulls", ct.c_void_p),
                ("on_device", I32), ("key_bound", I32)]


class sg_matches(ct.Structure):
    _fields_ = [("n", I64), ("trigger", ct.c_void_p), ("ts", ct.c_void_p), ("key", ct.c_void_p),
                ("group", ct.c_void_p), ("vals", ct.c_void_p), ("vnull", ct.c_void_p)]


class sg_match_columns(ct.Structure):
    _fields_ = [("trigger", ct.c_void_p), ("ts", ct.c_void_p), ("key", ct.c_void_p), ("group", ct.c_void_p),
                ("cols", ct.c_void_p * SG_MAX_SELECT), ("nulls", ct.c_void_p * SG_MAX_SELECT)]


SG_NODE_MAX_GPUS = 16


class sg_node_batch(ct.Structure):
    _fields_ = [("n", I64), ("base_index", U64), ("ts", ct.c_void_p), ("stream", ct.c_void_p),
                ("raw_key", ct.c_void_p), ("cols", ct.c_void_p), ("nulls", ct.c_void_p)]


class sg_node_stats(ct.Structure):
    _fields_ = [("total_ms", ct.c_double), ("reserve_ms", ct.c_double), ("route_ms", ct.c_double),
                ("merge_ms", ct.c_double), ("gpu_ms", ct.c_double * SG_NODE_MAX_GPUS),
                ("rows", I64), ("matches", I64), ("chunks", I64), ("chunk_rows", I64), ("h2d_bytes", I64),
                ("d2h_bytes", I64), ("shard_rows", I64 * SG_NODE_MAX_GPUS)]


class sg_match_records(ct.Structure):
    _fields_ = [("n", I64), ("record_bytes", I32), ("n_select", I32), ("base", ct.c_void_p)]


SG_MAX_KMARKS = 24


class sg_timing(ct.Structure):
    _fields_ = [("pred_ms", ct.c_float), ("partition_ms", ct.c_float), ("match_ms", ct.c_float),
                ("output_ms", ct.c_float), ("total_ms", ct.c_float), ("events", I64), ("matches", I64),
                ("spilled_units", I64), ("n_kernels", I32), ("kernel_ms", ct.c_float * SG_MAX_KMARKS),
                ("kernel_name", (ct.c_char * 32) * SG_MAX_KMARKS)]

    def kernels(self):
        """[(name, ms)] of the last push's marked kernels (HIP events on the launch stream)."""
        return [(self.kernel_name[k].value.decode(), self.kernel_ms[k]) for k in range(self.n_kernels)]


_lib = None


class SgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"siddhi_gpu error {code}: {msg}")
        self.code = code


def _one_hip_runtime():
    """Make the process's HIP runtime the one torch brings, before libsiddhi_gpu.so is loaded.

    torch's wheel ships its own libamdhip64 / libhsa-runtime64 (same sonames as /opt/rocm's).  Loaded first, torch's
    copies satisfy libsiddhi_gpu.so's dependencies by soname and the process has one HIP runtime.  Loaded the other
    way round (this library first, torch later) the dynamic linker maps BOTH runtimes and both HSA runtimes into the
    process, each opening the GPU on its own: after hundreds of engine handles had been opened and closed on the first
    one, torch's later initialisation found "No HIP GPUs are available" (r03 GPU suite).  A host without torch (the
    JNI binding) has one runtime anyway."""
    import sys
    if "torch" in sys.modules:
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_library(path: str = LIB_PATH):
    """Load libsiddhi_gpu.so; raises if it is not built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise RuntimeError(f"libsiddhi_gpu.so not built at {path}: run `make -C siddhi_amd/csrc` "
                               "or __graft_entry__.build()")
        _one_hip_runtime()
        lib = ct.CDLL(path)
        P = ct.c_void_p
        lib.sg_open.argtypes = [ct.c_int, P, P, ct.POINTER(P)]
        lib.sg_push.argtypes = [P, P]
        lib.sg_advance_time.argtypes = [P, I64, U64]
        lib.sg_pending.argtypes = [P, ct.POINTER(I64)]
        lib.sg_poll.argtypes = [P, P, I64, ct.POINTER(I64)]
        lib.sg_device_records.argtypes = [P, P]
        lib.sg_discard.argtypes = [P]
        lib.sg_flush.argtypes = [P]
        lib.sg_reset.argtypes = [P]
        lib.sg_set_stream.argtypes = [P, P]
        lib.sg_get_timing.argtypes = [P, P]
        lib.sg_close.argtypes = [P]
        lib.sg_snapshot.argtypes = [P, P, ct.c_size_t, ct.POINTER(ct.c_size_t)]
        lib.sg_restore.argtypes = [P, P, ct.c_size_t]
        lib.sg_host_alloc.argtypes = [ct.c_size_t, ct.POINTER(P)]
        lib.sg_host_free.argtypes = [P]
        lib.sg_poll_columns.argtypes = [P, P, I64, ct.POINTER(I64)]
        lib.sg_push_deliver.argtypes = [P, P, P, I64, ct.POINTER(I64)]
        lib.sg_router_open.argtypes = [ct.c_int, ct.c_int, ct.POINTER(P)]
        lib.sg_router_route.argtypes = [P, I64, P, P, P, P]
        lib.sg_router_keys.argtypes = [P, ct.POINTER(I64), I32, ct.POINTER(I64)]
        lib.sg_router_close.argtypes = [P]
        lib.sg_router_dense_ids.argtypes = [P, I32, P, I64]
        lib.sg_merge_order.argtypes = [ct.c_int, P, P, P, P, ct.c_int, P]
        lib.sg_node_open.argtypes = [ct.c_int, P, P, P, ct.c_int, I64, ct.POINTER(P)]
        lib.sg_node_push.argtypes = [P, P, P, I64, ct.POINTER(I64)]
        lib.sg_node_reset.argtypes = [P]
        lib.sg_node_stats_get.argtypes = [P, P]
        lib.sg_node_keys.argtypes = [P, ct.POINTER(I64)]
        lib.sg_node_close.argtypes = [P]
        lib.sg_node_set_key_dict.argtypes = [P, ct.c_int]
        lib.sg_node_last_error.argtypes = [P]
        lib.sg_node_last_error.restype = ct.c_char_p
        lib.sg_last_error.argtypes = [P]
        lib.sg_last_error.restype = ct.c_char_p
        lib.sg_version.restype = ct.c_char_p
        _lib = lib
    return _lib


def build_desc(nfa: L.FlatNFA) -> sg_nfa_desc:
    d = sg_nfa_desc()
    d.abi_version = SG_ABI_VERSION
    d.type = nfa.type
    d.within = nfa.within
    d.playback = nfa.playback
    d.partitioned = nfa.partitioned
    d.n_states = len(nfa.states)
    d.n_streams = max(1, max((s for s, _, _ in nfa.cols), default=0) + 1)
    d.n_cols = len(nfa.cols)
    d.n_ret = len(nfa.retained)
    d.n_select = len(nfa.select)
    code = []
    for i, st in enumerate(nfa.states):
        x = d.states[i]
        for f in ("kind", "stream", "is_start", "min_count", "max_count", "logical_type", "partner",
                  "next_state", "next_every", "within_every", "callback", "has_selector", "this_last",
                  "local"):
            setattr(x, f, int(getattr(st, f)))
        x.waiting_time = int(st.waiting_time)
        x.prog_off = len(code)
        x.prog_len = len(st.prog)
        code += st.prog
    d.shape = nfa.shape
    for k, v in enumerate(nfa.shape_args[:8]):
        d.shape_args[k] = int(v)
    d.shape_prog_off = len(code)
    d.shape_prog_len = len(nfa.shape_prog)
    code += nfa.shape_prog
    d.n_out = len(nfa.out_progs)
    for k, (w, t) in enumerate(zip(nfa.out_progs, nfa.out_types)):
        d.out_off[k] = len(code)
        d.out_len[k] = len(w)
        d.out_type[k] = L.TYPE_CODE[t]
        code += w
    if nfa.having_prog:
        d.having_off = len(code)
        d.having_len = len(nfa.having_prog)
        code += nfa.having_prog
    if len(code) > SG_MAX_CODE:
        raise L.LoweringError("predicate programs too long")
    d.code_len = len(code)
    for k, w in enumerate(code):
        d.code[k] = int(w)
    for s in range(SG_MAX_STREAMS):
        d.recv_of_stream[s] = -1
    for k, (s, r) in enumerate(sorted(nfa.receivers.items())):
        rr = d.receivers[k]
        rr.stream, rr.multi, rr.selector, rr.n = s, r.multi, r.selector, len(r.pres)
        for j, p in enumerate(r.pres):
            rr.pres[j] = p
        for j, p in enumerate(r.stab):
            rr.stab[j] = p
        d.recv_of_stream[s] = k
    d.n_init, d.n_reset, d.n_update, d.n_start = (len(nfa.init_order), len(nfa.reset_ops), len(nfa.update_ops),
                                                  len(nfa.start_ids))
    for k, v in enumerate(nfa.init_order):
        d.init_order[k] = v
    for k, v in enumerate(nfa.reset_ops):
        d.reset_ops[k] = v
    for k, v in enumerate(nfa.update_ops):
        d.update_ops[k] = v
    for k, v in enumerate(nfa.start_ids):
        d.start_ids[k] = v
    colidx = {}
    for c, (s, a, t) in enumerate(nfa.cols):
        d.col_type[c] = L.TYPE_CODE[t]
        d.col_stream[c] = s
        colidx[(s, a)] = c
    for r, (s, a, t) in enumerate(nfa.retained):
        d.ret_col[r] = colidx[(s, a)]
        d.ret_type[r] = L.TYPE_CODE[t]
    for k, (st, idx, slot, t) in enumerate(nfa.select):
        d.sel_state[k], d.sel_index[k], d.sel_ret[k], d.sel_type[k] = st, idx, slot, L.TYPE_CODE[t]
    d.n_sched = len(nfa.sched)
    for k, v in enumerate(nfa.sched):
        d.sched_state[k] = v
    return d


class Handle:
    """Thin RAII wrapper of one sg_handle."""

    def __init__(self, desc: sg_nfa_desc, device: int = 0, options: sg_options = None):
        self._pid = os.getpid()
        self.lib = load_library()
        self.h = ct.c_void_p()
        self.desc = desc
        self.opts = options if options is not None else sg_options()
        rc = self.lib.sg_open(device, ct.byref(desc), ct.byref(self.opts), ct.byref(self.h))
        if rc != 0:
            msg = self.lib.sg_last_error(self.h).decode() if self.h else ""
            if self.h:
                self.lib.sg_close(self.h)
            self.h = None
            raise SgError(rc, msg)

    def check(self, rc):
        if rc != 0:
            raise SgError(rc, self.lib.sg_last_error(self.h).decode())

    def push(self, b: sg_batch):
        self.check(self.lib.sg_push(self.h, ct.byref(b)))

    def advance_time(self, now: int, trigger_index: int):
        """Heartbeat: fire the timers due at `now` (sg_advance_time; one clock-only row)."""
        self.check(self.lib.sg_advance_time(self.h, int(now), int(trigger_index)))

    def pending(self) -> int:
        n = I64()
        self.check(self.lib.sg_pending(self.h, ct.byref(n)))
        return n.value

    def poll(self, nsel: int):
        n = self.pending()
        tr = np.zeros(n, np.uint64)
        ts = np.zeros(n, np.int64)
        ky = np.zeros(n, np.int32)
        gr = np.zeros(n, np.uint32)
        vals = np.zeros((n, max(nsel, 1)), np.int64)
        vn = np.zeros(n, np.uint32)
        if n:
            m = sg_matches(n, tr.ctypes.data, ts.ctypes.data, ky.ctypes.data, gr.ctypes.data, vals.ctypes.data,
                           vn.ctypes.data)
            got = I64()
            self.check(self.lib.sg_poll(self.h, ct.byref(m), n, ct.byref(got)))
        return tr, ts, ky, gr, vals[:, :nsel], vn

    def poll_columns(self, cols: "sg_match_columns", cap: int) -> int:
        """sg_poll_columns: up to cap pending matches as typed SoA columns into `cols` (host arrays)."""
        n = I64()
        self.check(self.lib.sg_poll_columns(self.h, ct.byref(cols), int(cap), ct.byref(n)))
        return n.value

    def push_deliver(self, b: sg_batch, cols: "sg_match_columns", cap: int) -> int:
        """sg_push_deliver: push a batch and receive its matches (and any pending ones) as SoA columns."""
        n = I64()
        self.check(self.lib.sg_push_deliver(self.h, ct.byref(b), ct.byref(cols), int(cap), ct.byref(n)))
        return n.value

    def device_records(self) -> sg_match_records:
        m = sg_match_records()
        self.check(self.lib.sg_device_records(self.h, ct.byref(m)))
        return m

    def timing(self) -> sg_timing:
        t = sg_timing()
        self.check(self.lib.sg_get_timing(self.h, ct.byref(t)))
        return t

    def reset(self):
        self.check(self.lib.sg_reset(self.h))

    def snapshot(self) -> bytes:
        """sg_snapshot: the handle's per-key state as an opaque blob (no undelivered matches allowed)."""
        size = ct.c_size_t()
        self.check(self.lib.sg_snapshot(self.h, None, 0, ct.byref(size)))
        buf = ct.create_string_buffer(max(size.value, 1))
        self.check(self.lib.sg_snapshot(self.h, buf, size.value, ct.byref(size)))
        return buf.raw[:size.value]

    def restore(self, blob: bytes):
        self.check(self.lib.sg_restore(self.h, blob, len(blob)))

    def discard(self):
        self.check(self.lib.sg_discard(self.h))

    def flush(self):
        self.check(self.lib.sg_flush(self.h))

    def close(self):
        if self.h:
            self.lib.sg_close(self.h)
            self.h = None

    def __del__(self):
        if getattr(self, "_pid", os.getpid()) != os.getpid():
            return   # (a forked child's copy: the parent owns the native object)
        try:
            self.close()
        except Exception:
            pass


def column_dtypes(nfa: L.FlatNFA):
    """numpy dtypes of the delivered output columns (sg_match_columns.cols): 4 or 8 bytes by Attribute.Type."""
    types = nfa.out_types if nfa.out_progs else [t for (_, _, _, t) in nfa.select]
    m = {"STRING": np.int32, "INT": np.int32, "BOOL": np.int32, "FLOAT": np.float32, "LONG": np.int64,
         "DOUBLE": np.float64}
    return [m[t] for t in types]


class ColumnSink:
    """Host arrays for SoA delivery (sg_match_columns), pinned when `pinned` (sg_host_alloc)."""

    def __init__(self, nfa: L.FlatNFA, cap: int, pinned: bool = True, fields=("trigger", "ts", "key", "group"),
                 nulls: bool = True):
        self.cap = cap
        self._keep = []

        def arr(dt):
            if pinned:
                p = PinnedArray(cap, dt)
                self._keep.append(p)
                return p.array
            return np.zeros(cap, dt)
        self.trigger = arr(np.uint64) if "trigger" in fields else None
        self.ts = arr(np.int64) if "ts" in fields else None
        self.key = arr(np.int32) if "key" in fields else None
        self.group = arr(np.uint32) if "group" in fields else None
        self.cols = [arr(dt) for dt in column_dtypes(nfa)]
        self.nulls = [arr(np.uint8) for _ in self.cols] if nulls else None
        s = sg_match_columns()
        for f in ("trigger", "ts", "key", "group"):
            a = getattr(self, f)
            setattr(s, f, a.ctypes.data if a is not None else None)
        for k, a in enumerate(self.cols):
            s.cols[k] = a.ctypes.data
            if self.nulls is not None:
                s.nulls[k] = self.nulls[k].ctypes.data
        self.struct = s


class Router:
    """The native host partition router (sg_router_*): dense first-seen key ids, shard and per-shard dense ids."""

    def __init__(self, n_shards: int = 1, threads: int = 0):
        self._pid = os.getpid()
        self.lib = load_library()
        self.r = ct.c_void_p()
        rc = self.lib.sg_router_open(n_shards, threads, ct.byref(self.r))
        if rc != 0:
            raise SgError(rc, "sg_router_open failed")

    def route(self, raw: np.ndarray, dense=None, shard=None, local=None):
        raw = np.ascontiguousarray(raw, np.int64)
        ptr = lambda a: a.ctypes.data if a is not None else None   # noqa: E731
        rc = self.lib.sg_router_route(self.r, len(raw), raw.ctypes.data, ptr(dense), ptr(shard), ptr(local))
        if rc != 0:
            raise SgError(rc, "sg_router_route failed")

    def keys(self, shard: int = -1):
        n, sk = I64(), I64()
        self.lib.sg_router_keys(self.r, ct.byref(n), shard, ct.byref(sk))
        return n.value, sk.value

    def close(self):
        if self.r:
            self.lib.sg_router_close(self.r)
            self.r = None

    def __del__(self):
        if getattr(self, "_pid", os.getpid()) != os.getpid():
            return   # (a forked child's copy: the parent owns the native object)
        try:
            self.close()
        except Exception:
            pass


def merge_order(triggers, groups=None, keys=None, threads: int = 16) -> np.ndarray:
    """sg_merge_order: the node's delivery order of several match runs (each in delivery order) as indices into
    their concatenation -- by (trigger, phase, dense key), ties in run order."""
    lib = load_library()
    n = len(triggers)
    tr = [np.ascontiguousarray(t, np.uint64) for t in triggers]
    gr = None if groups is None else [np.ascontiguousarray(g, np.uint32) for g in groups]
    ky = None if keys is None else [np.ascontiguousarray(k, np.int32) for k in keys]
    lens = np.array([len(t) for t in tr], np.int64)
    P = ct.c_void_p
    ptrs = lambda arrs: None if arrs is None else ct.cast((P * max(n, 1))(*[a.ctypes.data for a in arrs]), P)  # noqa
    out = np.zeros(int(lens.sum()), np.int64)
    rc = lib.sg_merge_order(n, lens.ctypes.data, ptrs(tr), ptrs(gr), ptrs(ky), threads, out.ctypes.data)
    if rc != 0:
        raise SgError(rc, "sg_merge_order failed")
    return out


class Node:
    """The node pipeline (sg_node_*): raw host rows -> native router -> every GPU of the node (one thread each,
    chunks with H2D / kernels / D2H overlapped) -> merged matches in delivery order."""

    def __init__(self, desc: sg_nfa_desc, n_gpus: int = 1, devices=None, options: sg_options = None,
                 threads: int = 16, chunk_rows: int = 0):
        self._pid = os.getpid()
        self.lib = load_library()
        self.n = ct.c_void_p()
        self.desc = desc
        self.opts = options if options is not None else sg_options()
        devs = (ct.c_int * n_gpus)(*(devices if devices is not None else range(n_gpus)))
        rc = self.lib.sg_node_open(n_gpus, devs, ct.byref(desc), ct.byref(self.opts), threads, chunk_rows,
                                   ct.byref(self.n))
        if rc != 0:
            raise SgError(rc, "sg_node_open failed")

    def check(self, rc):
        if rc != 0:
            raise SgError(rc, self.lib.sg_node_last_error(self.n).decode())

    def push(self, b: sg_node_batch, cols: "sg_match_columns", cap: int) -> int:
        n = I64()
        self.check(self.lib.sg_node_push(self.n, ct.byref(b), ct.byref(cols), int(cap), ct.byref(n)))
        return n.value

    def stats(self) -> dict:
        st = sg_node_stats()
        self.check(self.lib.sg_node_stats_get(self.n, ct.byref(st)))
        g = int(self.desc_gpus) if hasattr(self, "desc_gpus") else SG_NODE_MAX_GPUS
        return {"total_ms": st.total_ms, "reserve_ms": st.reserve_ms, "route_ms": st.route_ms,
                "merge_ms": st.merge_ms, "gpu_ms": [st.gpu_ms[k] for k in range(g)], "rows": st.rows,
                "matches": st.matches, "chunks": st.chunks, "chunk_rows": st.chunk_rows, "h2d_bytes": st.h2d_bytes,
                "d2h_bytes": st.d2h_bytes, "shard_rows": [st.shard_rows[k] for k in range(g)]}

    def keys(self) -> int:
        n = I64()
        self.check(self.lib.sg_node_keys(self.n, ct.byref(n)))
        return n.value

    def reset(self):
        self.check(self.lib.sg_node_reset(self.n))

    def set_key_dict(self, mode: int):
        """0 auto, 1 host router, 2 device dictionary (before the first push of a stream)."""
        self.check(self.lib.sg_node_set_key_dict(self.n, int(mode)))

    def close(self):
        if self.n:
            self.lib.sg_node_close(self.n)
            self.n = None

    def __del__(self):
        if getattr(self, "_pid", os.getpid()) != os.getpid():
            return   # (a forked child's copy: the parent owns the native object)
        try:
            self.close()
        except Exception:
            pass


def make_node_batch(n, base_index, ts, stream, raw_key, cols, nulls, keep):
    """Assemble an sg_node_batch from raw host pointers (ints; 0 = absent)."""
    ncol = len(cols)
    carr = (ct.c_void_p * max(ncol, 1))(*[(c if c else None) for c in cols])
    narr = (ct.c_void_p * max(ncol, 1))(*[(x if x else None) for x in nulls])
    keep += [carr, narr]
    has_nul = any(bool(x) for x in nulls)
    return sg_node_batch(n, base_index, ts or None, stream or None, raw_key or None, ct.cast(carr, ct.c_void_p),
                         ct.cast(narr, ct.c_void_p) if has_nul else None)


class PinnedArray:
    """A numpy array over pinned host memory from sg_host_alloc (freed with the object)."""

    def __init__(self, n: int, dtype):
        self._pid = os.getpid()
        self.lib = load_library()
        self.p = ct.c_void_p()
        dt = np.dtype(dtype)
        rc = self.lib.sg_host_alloc(max(n, 1) * dt.itemsize, ct.byref(self.p))
        if rc != 0:
            raise SgError(rc, "sg_host_alloc failed")
        buf = (ct.c_char * (max(n, 1) * dt.itemsize)).from_address(self.p.value)
        self.array = np.frombuffer(buf, dtype=dt, count=n)

    def __del__(self):
        if getattr(self, "_pid", os.getpid()) != os.getpid():
            return   # (a forked child's copy: the parent owns the pinned memory)
        if getattr(self, "p", None) and self.p.value:
            self.array = None
            self.lib.sg_host_free(self.p)
            self.p = ct.c_void_p()


def make_batch(n, base_index, ts, stream, key, cols, nulls, on_device, key_bound=0, keep=None, index=0):
    """Assemble an sg_batch from raw pointers (ints); `keep` collects ctypes arrays to keep alive."""
    ncol = len(cols)
    carr = (ct.c_void_p * max(ncol, 1))(*[c for c in cols])
    narr = (ct.c_void_p * max(ncol, 1))(*[(x if x else None) for x in nulls])
    if keep is not None:
        keep += [carr, narr]
    return sg_batch(n, base_index, ts, stream, key, index or None, ct.cast(carr, ct.c_void_p),
                    ct.cast(narr, ct.c_void_p), on_device, key_bound)


class GpuEngine:
    """Engine interface (see siddhi_amd/runtime.py) on the MI355X kernels."""

    def __init__(self, ctx: L.QueryContext, device: int = 0, force_general: bool = False, pool: int = 0,
                 no_carry: bool = False, ring_cap: int = 0, chunk_rows: int = 0, walker_only: bool = False,
                 ingress_rows: int = 0, partition_sort: int = 0, partial_lanes: int = 0, no_grow: bool = False,
                 max_lateness_ms: int = -1):
        self.ctx = ctx
        self.nfa = L.lower(ctx)
        self.desc = build_desc(self.nfa)
        opts = sg_options()
        opts.force_general = 1 if force_general else 0
        opts.no_carry = 1 if no_carry else 0
        opts.ring_cap = ring_cap
        opts.chunk_rows = chunk_rows
        opts.walker_only = 1 if walker_only else 0
        opts.ingress_rows = ingress_rows
        opts.partition_sort = partition_sort
        opts.partial_lanes = partial_lanes
        opts.no_grow = 1 if no_grow else 0
        if max_lateness_ms >= 0:   # (sg_options.bounded_lateness: pending partials that can never emit are not carried)
            opts.bounded_lateness = 1
            opts.max_lateness_ms = max_lateness_ms
        if pool:
            opts.pool_partials = opts.pool_events = opts.pool_chain = opts.list_cap = pool
        self.handle = Handle(self.desc, device, opts)
        self.nsel = len(self.nfa.out_progs) or len(self.nfa.select)

    def push(self, b):
        import numpy as np
        keep = []
        ts = np.ascontiguousarray(b.ts, np.int64)
        st = None if b.stream is None else np.ascontiguousarray(b.stream, np.int32)   # None: every row stream 0
        ky = np.ascontiguousarray(b.key, np.int32)
        cols = [np.ascontiguousarray(c) for c in b.cols]
        keep += [ts, st, ky] + cols + [x for x in b.nulls if x is not None]
        kb = int(ky.max()) + 1 if len(ky) and ky.max() >= 0 else 1
        ix = 0
        if getattr(b, "index", None) is not None:
            ixa = np.ascontiguousarray(b.index, np.uint64)
            keep.append(ixa)
            ix = ixa.ctypes.data
        sb = make_batch(b.n, b.base_index, ts.ctypes.data, 0 if st is None else st.ctypes.data, ky.ctypes.data,
                        [c.ctypes.data for c in cols], [(x.ctypes.data if x is not None else 0) for x in b.nulls],
                        0, kb, keep, index=ix)
        self.handle.push(sb)

    def fetch(self):
        from .runtime import Outputs
        tr, ts, ky, gr, vals, vn = self.handle.poll(self.nsel)
        vnull = np.zeros((len(tr), self.nsel), np.uint8)
        for k in range(self.nsel):
            vnull[:, k] = (vn >> np.uint32(k)) & np.uint32(1)
        return Outputs(tr, ts, ky, gr, vals, vnull)

    def snapshot(self) -> bytes:
        return self.handle.snapshot()

    def restore(self, blob: bytes):
        self.handle.restore(blob)

    def close(self):
        self.handle.close()
