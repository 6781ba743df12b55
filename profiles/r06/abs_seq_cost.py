"""Cost of the absence route's exact sequential pass (k_abs_seq, csrc/absent.hip) at C4's full size.

C4 (BASELINE configs[3]): 10M S events over 10k ids, `every e1=S -> not S[id==e1.id] for 5 sec` under @app:playback.
The stream is pushed as two 5M-row pushes (state carried) and the final Tick fires every remaining timer.  Variants:
every timestamp non-decreasing (the bench's stream), and L rows of the FIRST push moved 2 s back in time (late rows:
the push takes the exact sequential pass, and so does every later push while the carried timer FIFO is not sorted
and above the clock).  Prints one JSON line per variant: wall ms per push (host sync after each), the route's kernel
times (sg_timing), matches.  Usage: python profiles/r06/abs_seq_cost.py [late counts, default 0,1,100]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from siddhi_amd import _native as N  # noqa: E402
from siddhi_amd import synth  # noqa: E402


def run(late, n=10_000_000, ids=10_000, pushes=2):
    dev = torch.device("cuda", 0)
    g, key, cols = bench.synth_columns("C4", 0, n, ids, 1, dev)
    ts = g["ts"].clone()
    if late:
        rng = np.random.default_rng(5)
        pos = torch.from_numpy(np.sort(rng.choice(np.arange(1000, n // pushes), late, replace=False))).to(dev)
        ts[pos] -= 2000
    torch.cuda.synchronize()
    h, _ = bench.make_handle("C4", no_carry=0)
    stream = torch.cuda.current_stream()
    h.check(h.lib.sg_set_stream(h.h, stream.cuda_stream))
    step = n // pushes
    rows = []
    matches = 0
    for p in range(pushes):
        lo = p * step
        keep = []
        b = N.make_batch(step, lo, ts.data_ptr() + 8 * lo, 0, key.data_ptr() + 4 * lo,
                         [c.data_ptr() + c.element_size() * lo for c in cols], [0] * len(cols), 1, 1, keep)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.push(b)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        t = h.timing()
        rows.append({"push": p, "wall_ms": round(ms, 3), "kernels_ms": {k: round(v, 3) for k, v in t.kernels()}})
    tick = int(synth.T0 + (n - 1) + 5001 + 5000)
    t0 = time.perf_counter()
    h.advance_time(tick, n)
    torch.cuda.synchronize()
    rows.append({"tick_wall_ms": round((time.perf_counter() - t0) * 1e3, 3)})
    matches = h.pending()
    h.close()
    return {"late_rows": late, "events": n, "ids": ids, "pushes": pushes, "matches": matches, "per_push": rows}


if __name__ == "__main__":
    lates = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,100").split(",")]
    run(0, n=1_000_000)   # warm-up (module load, workspace)
    for late in lates:
        print(json.dumps(run(late)), flush=True)
