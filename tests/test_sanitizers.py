"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the host-side C++: the CPU oracle
(oracle/oracle.cpp), the host build of the GPU's per-key machine (tests/host_interp/harness.cpp over
siddhi_amd/csrc/interp.h) and the C-ABI partition router (siddhi_amd/csrc/router.cpp).

Engine calls of the reference KATs and of synthetic config batches are recorded from Python, replayed by standalone
sanitizer-built executables (tests/sanitize/driver.cpp: no preloading, the runtime is linked in) and must (a) finish
without a sanitizer report and (b) produce exactly the unsanitised build's outputs.  GPU code is not covered here:
GPU sanitizers are unavailable on this pool."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import synth_batch
from ref_kats import REF_KATS, run_ref_kat
from siddhi_amd import lowering as L
from siddhi_amd import synth
from siddhi_amd.runtime import Outputs

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
import sys  # noqa: E402
sys.path.insert(0, os.path.join(HERE, "host_interp"))
from host_engine import HostInterpEngine  # noqa: E402
SAN = os.path.join(HERE, "sanitize")
BUILD = os.path.join(SAN, "_build")
FLAGS = ["-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
         "-fno-sanitize-recover=undefined", "-Wall", "-Wno-unused-function"]
TARGETS = {
    "san_oracle": (["-DSAN_ORACLE"], [os.path.join(ROOT, "oracle", "oracle.cpp")]),
    "san_interp": (["-DSAN_INTERP"], [os.path.join(HERE, "host_interp", "harness.cpp")]),
    "san_router": (["-DSAN_ROUTER", "-pthread"], [os.path.join(ROOT, "siddhi_amd", "csrc", "router.cpp")]),
}
DEPS = [os.path.join(SAN, "driver.cpp"), os.path.join(ROOT, "include", "siddhi_gpu.h"),
        os.path.join(ROOT, "siddhi_amd", "csrc", "interp.h"), os.path.join(ROOT, "siddhi_amd", "csrc", "sg_device.h")]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _build(name):
    exe = os.path.join(BUILD, name)
    defs, srcs = TARGETS[name]
    deps = DEPS + srcs
    if not os.path.exists(exe) or any(os.path.getmtime(exe) < os.path.getmtime(d) for d in deps):
        import fcntl
        os.makedirs(BUILD, exist_ok=True)
        with open(exe + ".lock", "w") as lk:   # parallel test workers: one builds, the others wait for it
            fcntl.flock(lk, fcntl.LOCK_EX)
            if not os.path.exists(exe) or any(os.path.getmtime(exe) < os.path.getmtime(d) for d in deps):
                tmp = f"{exe}.{os.getpid()}.tmp"
                subprocess.run(["g++"] + FLAGS + defs + [os.path.join(SAN, "driver.cpp")] + srcs + ["-o", tmp],
                               check=True)
                os.replace(tmp, exe)
    return exe


def _run(exe, args):
    p = subprocess.run([exe] + args, env=ENV, capture_output=True, text=True, timeout=600)
    report = "ERROR: AddressSanitizer" in p.stderr or "runtime error:" in p.stderr or "LeakSanitizer" in p.stderr
    assert p.returncode == 0 and not report, p.stderr[-4000:]


class _Recorder:
    """Engine wrapper recording every push (deep copies) and the outputs of the wrapped engine."""
    log = []

    def __init__(self, inner, ctx, image):
        self.inner, self.image, self.nsel = inner, image, len(ctx.query.select)
        self.batches, self.outs = [], []
        _Recorder.log.append(self)

    def push(self, b):
        self.batches.append(b)
        self.inner.push(b)

    def fetch(self):
        o = self.inner.fetch()
        self.outs.append(o)
        return o

    def close(self):
        self.inner.close()

    def output(self):
        f = ("trigger", "ts", "key", "group", "vals", "vnull")
        return Outputs(*[np.concatenate([getattr(o, x) for o in self.outs]) if self.outs else np.zeros(0) for x in f])


def _oracle_rec(ctx):
    return _Recorder(OracleEngine(ctx), ctx, np.array(L.oracle_image(ctx), np.int64))


def _interp_rec(ctx):
    e = HostInterpEngine(ctx)
    raw = bytes(e.desc)
    raw += b"\0" * (-len(raw) % 8)
    return _Recorder(e, ctx, np.frombuffer(raw, np.int64).copy())


def _write_cases(path, recs):
    with open(path, "wb") as f:
        f.write(b"SGCASE01")
        for r in recs:
            f.write(struct.pack("<q", len(r.image)))
            f.write(r.image.astype("<i8").tobytes())
            cols = r.batches[0].cols if r.batches else []
            f.write(struct.pack("<qq", r.nsel, len(cols)))
            for c in cols:
                f.write(struct.pack("<q", np.asarray(c).dtype.itemsize))
            f.write(struct.pack("<q", len(r.batches)))
            for b in r.batches:
                idx = getattr(b, "index", None)
                f.write(struct.pack("<qQq", b.n, b.base_index, 0 if idx is None else 1))
                f.write(np.ascontiguousarray(b.ts, "<i8").tobytes())
                st = b.stream if b.stream is not None else np.zeros(b.n, np.int32)
                f.write(np.ascontiguousarray(st, "<i4").tobytes())
                f.write(np.ascontiguousarray(b.key, "<i4").tobytes())
                if idx is not None:
                    f.write(np.ascontiguousarray(idx, "<u8").tobytes())
                for c, nl in zip(b.cols, b.nulls):
                    f.write(np.ascontiguousarray(c).tobytes())
                    f.write(struct.pack("<q", 0 if nl is None else 1))
                    if nl is not None:
                        f.write(np.ascontiguousarray(nl, np.uint8).tobytes())


def _read_outputs(path, recs, interp):
    data = open(path, "rb").read()
    pos = 0

    def take(dt, count):
        nonlocal pos
        a = np.frombuffer(data, dt, count, pos)
        pos += a.nbytes
        return a

    outs = []
    for r in recs:
        (n,) = struct.unpack_from("<q", data, pos)
        pos += 8
        tr, ts, ky, gr = take("<u8", n), take("<i8", n), take("<i4", n), take("<u4", n)
        vals = take("<i8", n * r.nsel).reshape(n, r.nsel)
        if interp:
            vn32 = take("<u4", n)
            vn = np.stack([(vn32 >> np.uint32(k)) & 1 for k in range(r.nsel)], axis=1).astype(np.uint8) if r.nsel \
                else np.zeros((n, 0), np.uint8)
        else:
            vn = take("<u1", n * r.nsel).reshape(n, r.nsel)
        outs.append(Outputs(tr, ts, ky, gr, vals, vn))
    assert pos == len(data)
    return outs


def _same(a, b):
    assert len(a.trigger) == len(b.trigger)
    for f in ("trigger", "ts", "key", "group"):
        assert np.array_equal(np.asarray(getattr(a, f)).astype(np.int64), np.asarray(getattr(b, f)).astype(np.int64)), f
    if len(a.trigger):
        na = np.asarray(a.vnull).astype(bool)
        assert np.array_equal(na, np.asarray(b.vnull).astype(bool))
        assert np.array_equal(np.where(na, 0, a.vals), np.where(na, 0, b.vals))


def _replay(tmp_path, exe_name, recs, interp):
    exe = _build(exe_name)
    cases, out = str(tmp_path / "cases.bin"), str(tmp_path / "out.bin")
    _write_cases(cases, recs)
    _run(exe, [cases, out])
    for r, o in zip(recs, _read_outputs(out, recs, interp)):
        _same(o, r.output())


def _kat_recordings(factory):
    _Recorder.log = []
    for case in REF_KATS:
        run_ref_kat(case, factory)
    recs, _Recorder.log = _Recorder.log, []
    return [r for r in recs if r.batches]


@pytest.mark.parametrize("which", ["oracle", "interp"])
def test_sanitized_reference_kats(tmp_path, which):
    """All transcribed reference KATs (tests/golden/ref_kats.json) replayed under ASan+UBSan."""
    recs = _kat_recordings(_oracle_rec if which == "oracle" else _interp_rec)
    assert len(recs) >= 300
    _replay(tmp_path, "san_" + which, recs, which == "interp")


@pytest.mark.parametrize("which", ["oracle", "interp"])
def test_sanitized_config_batches(tmp_path, which):
    """Synthetic config batches (closed-form and general-machine shapes, multi-push carry) under ASan+UBSan."""
    from parity_util import run_engine
    _Recorder.log = []
    fac = _oracle_rec if which == "oracle" else _interp_rec
    cfgs = [("C2", 20_000, 500), ("C3", 8_000, 20), ("C3b", 8_000, 20), ("C3c", 8_000, 20)]
    if which == "oracle":   # (closed-form shapes whose per-key lists exceed the host machine's fixed pools)
        cfgs += [("C1", 3_000, 1), ("C2", 20_000, 50), ("C4", 6_000, 100)]
    for cfg, n, keys in cfgs:
        b = synth_batch(cfg, 0, n, keys=keys, rate=20)
        half = n // 2
        from siddhi_amd.runtime import Batch
        parts = [Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi], [c[lo:hi] for c in b.cols],
                       [None] * len(b.cols)) for lo, hi in ((0, half), (half, n))]
        run_engine(fac, synth.QUERIES[cfg], parts)
    recs, _Recorder.log = _Recorder.log, []
    _replay(tmp_path, "san_" + which, recs, which == "interp")


def test_sanitized_router(tmp_path):
    """The native partition router under ASan+UBSan with 4 worker threads: dense ids, shards and per-shard ids
    equal the unsanitised library's."""
    from siddhi_amd._native import Router
    exe = _build("san_router")
    rng = np.random.default_rng(3)
    calls = [rng.integers(-5, 50_000, size=n).astype(np.int64) for n in (1, 70_000, 300_000, 5)]
    inp, out = str(tmp_path / "raw.bin"), str(tmp_path / "route.bin")
    with open(inp, "wb") as f:
        for c in calls:
            f.write(struct.pack("<q", len(c)) + c.tobytes())
    _run(exe, ["3", "4", inp, out])
    data = open(out, "rb").read()
    r = Router(3, 4)
    pos = 0
    for c in calls:
        n = len(c)
        dense, shard, local = (np.zeros(n, np.int32) for _ in range(3))
        r.route(c, dense, shard, local)
        got = [np.frombuffer(data, "<i4", n, pos + k * 4 * n) for k in range(3)]
        pos += 12 * n
        assert np.array_equal(got[0], dense) and np.array_equal(got[1], shard) and np.array_equal(got[2], local)
    r.close()
