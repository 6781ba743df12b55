"""Diagnostic: device-memory delta per engine route / node after repeated open-push-close cycles."""
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
def free():
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipDeviceSynchronize()
    hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
    return f.value
ROUTES = [('C1', 3000, 1, 1), ('C2', 4000, 50, 10), ('C3b', 4000, 40, 10), ('C3c', 4000, 40, 10),
          ('C4', 3000, 100, 1), ('PP', 4000, 40, 10)]
for c, n, k, r in ROUTES:
    b = synth_batch(c, 0, n, keys=k, rate=r)
    run_engine(N.GpuEngine, synth.QUERIES[c], [b]); gc.collect()
    for rnd in range(3):
        f0 = free(); v0 = status('VmSize'); r0 = status('VmRSS')
        for i in range(40):
            run_engine(N.GpuEngine, synth.QUERIES[c], [b])
        gc.collect()
        f1 = free()
        print(f"{c} round {rnd}: {(f0 - f1) / 2**20:.2f} MiB device, VmSize +{status('VmSize') - v0} MiB, RSS +{status('VmRSS') - r0} MiB over 40 handles", flush=True)
# bare open/close
nfa = lower(context(synth.QUERIES['C2'])); desc = N.build_desc(nfa)
for rnd in range(2):
    f0 = free(); v0 = status('VmSize'); r0 = status('VmRSS')
    for i in range(200):
        h = N.Handle(desc, 0); h.close()
    print(f"open/close only x200: {(f0 - free()) / 2**20:.2f} MiB, VmSize +{status('VmSize') - v0}, RSS +{status('VmRSS') - r0}", flush=True)
for rnd in range(2):
    v0 = status('VmSize'); r0 = status('VmRSS')
    for i in range(50):
        p = N.PinnedArray(1 << 20, np.int64); del p
    print(f"pinned 8MiB x50: VmSize +{status('VmSize') - v0}, RSS +{status('VmRSS') - r0}", flush=True)
b2 = synth_batch('C2', 0, 20000, keys=200, rate=10)
ts = np.ascontiguousarray(b2.ts, np.int64); raw = synth.raw_symbols(b2.key).astype(np.int64)
cols = [np.ascontiguousarray(x) for x in b2.cols]
for G in (1, 2):
    for it in range(3):
        f0 = free()
        for i in range(5):
            keep = [ts, raw] + cols
            nb = N.make_node_batch(b2.n, 0, ts.ctypes.data, 0, raw.ctypes.data, [x.ctypes.data for x in cols], [0] * len(cols), keep)
            node = N.Node(desc, n_gpus=G, devices=[0] * G, threads=4, chunk_rows=6000)
            sink = N.ColumnSink(nfa, 40000, pinned=True)
            node.push(nb, sink.struct, sink.cap)
            node.close(); del sink; gc.collect()
        print(f"node G={G} round {it}: {(f0 - free()) / 2**20:.2f} MiB lost over 5 nodes, VmSize {status('VmSize')}, RSS {status('VmRSS')}", flush=True)
