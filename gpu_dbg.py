import sys, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import torch, numpy as np
from siddhi_amd import _native as N, lowering as L, synth
from parity_util import context
dev = torch.device("cuda", 0)
for n, keys in ((100_000, 500), (1_000_000, 10_000), (10_000_000, 10_000), (100_000_000, 10_000)):
    g = synth.generate_torch("C3b", 0, n, dev, keys=keys, rate=1000)
    key = g["key"].to(torch.int32)
    cols = [g["id"], key, g["v"], g["w"]]
    torch.cuda.synchronize()
    nfa = L.lower(context(synth.QUERIES["C3b"]))
    opts = N.sg_options()
    opts.no_carry = 1
    h = N.Handle(N.build_desc(nfa), device=0, options=opts)
    keep = []
    b = N.make_batch(n, 0, g["ts"].data_ptr(), 0, key.data_ptr(), [c.data_ptr() for c in cols], [0] * 4, 1, keys, keep)
    h.push(b)
    t = h.timing()
    print(n, keys, t.matches, [(nm, round(ms, 3)) for nm, ms in t.kernels()], flush=True)
    h.close()
