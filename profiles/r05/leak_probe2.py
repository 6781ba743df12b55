"""Diagnostic: the leak test's own sequence (one handle per route + one node per pipeline, then 500 handles and 20
nodes) with a snapshot after every step group, to find which step holds memory."""
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
def status(k):
    for line in open('/proc/self/status'):
        if line.startswith(k + ':'):
            return int(line.split()[1]) // 1024
    return 0
def free(sync):
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    if sync: hip.hipDeviceSynchronize()
    hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
    return f.value >> 20
def snap(tag):
    gc.collect()
    print(f"{tag}: free(no sync) {free(False)} MiB free(sync) {free(True)} MiB VmSize {status('VmSize')} RSS {status('VmRSS')} "
          f"threads {len(os.listdir('/proc/self/task'))}", flush=True)
ROUTES = [('C1', 3000, 1, 1), ('C2', 4000, 50, 10), ('C3b', 4000, 40, 10), ('C3c', 4000, 40, 10),
          ('C4', 3000, 100, 1), ('PP', 4000, 40, 10)]
batches = {c: synth_batch(c, 0, n, keys=k, rate=r) for c, n, k, r in ROUTES}
def one_handle(c):
    return len(run_engine(N.GpuEngine, synth.QUERIES[c], [batches[c]]))
nfa = lower(context(synth.QUERIES['C2'])); desc = N.build_desc(nfa)
b2 = synth_batch('C2', 0, 20000, keys=200, rate=10)
ts = np.ascontiguousarray(b2.ts, np.int64); raw = synth.raw_symbols(b2.key).astype(np.int64)
cols = [np.ascontiguousarray(x) for x in b2.cols]
def one_node(G):
    keep = [ts, raw] + cols
    nb = N.make_node_batch(b2.n, 0, ts.ctypes.data, 0, raw.ctypes.data, [x.ctypes.data for x in cols], [0] * len(cols), keep)
    node = N.Node(desc, n_gpus=G, devices=[0] * G, threads=4, chunk_rows=6000)
    sink = N.ColumnSink(nfa, 40000, pinned=True)
    got = node.push(nb, sink.struct, sink.cap)
    node.close()
    del sink
    return got
snap("start")
for c, *_ in ROUTES:
    one_handle(c)
    snap(f"warm {c}")
one_node(1); snap("warm node G=1")
one_node(2); snap("warm node G=2")
for rnd in range(3):
    for c, *_ in ROUTES:
        for i in range(28):
            one_handle(c)
        snap(f"round {rnd} {c} x28")
for i in range(10):
    one_node(1 + i % 2)
    snap(f"node {i} G={1 + i % 2}")
