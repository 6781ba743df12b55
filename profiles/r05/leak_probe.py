"""Diagnostic: host / device memory per engine route and per node over repeated open-push-close rounds.
Prints VmSize / RSS deltas and glibc heap in use (mallinfo2) so arena retention and real leaks can be told apart."""
import ctypes, gc, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]
from siddhi_amd import _native as N
N.load_library()
from parity_util import run_engine, synth_batch, context
from siddhi_amd import synth
from siddhi_amd.lowering import lower
import numpy as np
hip = ctypes.CDLL('libamdhip64.so.7')
libc = ctypes.CDLL('libc.so.6')
class MI2(ctypes.Structure):
    _fields_ = [(f, ctypes.c_size_t) for f in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks", "fsmblks",
                                               "uordblks", "fordblks", "keepcost")]
libc.mallinfo2.restype = MI2
def status(k):
    for line in open('/proc/self/status'):
        if line.startswith(k + ':'):
            return int(line.split()[1]) // 1024
    return 0
def free():
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipDeviceSynchronize()
    hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
    return f.value
def snap():
    gc.collect()
    m = libc.mallinfo2()
    return free(), status('VmSize'), status('VmRSS'), (m.uordblks + m.hblkhd) >> 20, m.arena >> 20
def report(tag, a, b):
    print(f"{tag}: device {(a[0] - b[0]) / 2**20:+.1f} MiB, VmSize {b[1] - a[1]:+d}, RSS {b[2] - a[2]:+d}, "
          f"heap in use {b[3] - a[3]:+d}, arena {b[4] - a[4]:+d} MiB", flush=True)
ROUTES = [('C1', 3000, 1, 1), ('C2', 4000, 50, 10), ('C3b', 4000, 40, 10), ('C3c', 4000, 40, 10),
          ('C4', 3000, 100, 1), ('PP', 4000, 40, 10)]
for c, n, k, r in ROUTES:
    b = synth_batch(c, 0, n, keys=k, rate=r)
    run_engine(N.GpuEngine, synth.QUERIES[c], [b])
    for rnd in range(3):
        s0 = snap()
        for i in range(40):
            run_engine(N.GpuEngine, synth.QUERIES[c], [b])
        report(f"{c} round {rnd} (40 handles)", s0, snap())
nfa = lower(context(synth.QUERIES['C2'])); desc = N.build_desc(nfa)
for rnd in range(2):
    s0 = snap()
    for i in range(200):
        h = N.Handle(desc, 0); h.close()
    report(f"open/close x200 round {rnd}", s0, snap())
for rnd in range(2):
    s0 = snap()
    for i in range(50):
        p = N.PinnedArray(1 << 20, np.int64); del p
    report(f"pinned 8MiB x50 round {rnd}", s0, snap())
b2 = synth_batch('C2', 0, 20000, keys=200, rate=10)
ts = np.ascontiguousarray(b2.ts, np.int64); raw = synth.raw_symbols(b2.key).astype(np.int64)
cols = [np.ascontiguousarray(x) for x in b2.cols]
for G in (1, 2, 1, 2):
    for it in range(3):
        s0 = snap()
        for i in range(5):
            keep = [ts, raw] + cols
            nb = N.make_node_batch(b2.n, 0, ts.ctypes.data, 0, raw.ctypes.data, [x.ctypes.data for x in cols], [0] * len(cols), keep)
            node = N.Node(desc, n_gpus=G, devices=[0] * G, threads=4, chunk_rows=6000)
            sink = N.ColumnSink(nfa, 40000, pinned=True)
            node.push(nb, sink.struct, sink.cap)
            node.close(); del sink
        report(f"node G={G} round {it} (5 nodes)", s0, snap())
