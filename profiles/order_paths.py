"""Partial-lane delivery order, the three paths side by side on one GPU (csrc/partial.hip, sg_partial_push):
one composed 64-bit key (default where it fits), the trigger-row sort plus in-place tie runs (k_pp_ties: the default
where it does not), and the three LSD radix sorts (the fallback for runs of more than 256 matches).  Forced through
sg_options.partial_lanes = 0 / 1 / 2; prints the `match_order` stage time of each and checks the outputs agree."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity_util import context, dense_first_seen   # noqa: E402
from siddhi_amd import synth   # noqa: E402
from siddhi_amd._native import GpuEngine   # noqa: E402
from siddhi_amd.runtime import Batch   # noqa: E402

Q = ("define stream S (id long, symbol string, v int, w int); partition with (symbol of S) begin @info(name='q') "
     "from every e1=S[v>80] -> e2=S[v>e1.v] -> e3=S[w>e1.w] -> e4=S[v<e1.v] within 1 hour "
     "select e1.id as i1, e2.id as i2, e3.id as i3, e4.id as i4 insert into M; end;")


def small_batch(n, keys, vmax, rate, seed):   # the shape of tests/test_partial_lanes.py's batches
    rng = np.random.default_rng(seed)
    ts = (synth.T0 + np.arange(n) // rate).astype(np.int64)
    key = dense_first_seen(rng.integers(0, keys, n).astype(np.int64)).astype(np.int32)
    v = rng.integers(0, vmax, n).astype(np.int32)
    w = rng.integers(0, vmax, n).astype(np.int32)
    return Batch(n, 0, ts, np.zeros(n, np.int32), key, [np.arange(n, dtype=np.int64), key, v, w], [None] * 4)


def main(n=int(os.environ.get("ORDER_ROWS", 20_000_000)), keys=4000, reps=3):
    b = small_batch(n, keys, 100, 20, seed=11)
    res, ref = {}, None
    for order in (0, 1, 2):
        eng = GpuEngine(context(Q), partial_lanes=order)
        best = None
        for r in range(reps):
            eng.handle.reset()
            eng.push(b)
            t = dict(eng.handle.timing().kernels())
            best = t if best is None or t["match_order"] < best["match_order"] else best
            out = eng.fetch()
        eng.close()
        if ref is None:
            ref = out
        same = all(np.array_equal(getattr(out, f), getattr(ref, f)) for f in ("trigger", "ts", "key", "vals"))
        res[order] = {"match_order_ms": round(best["match_order"], 3), "partial_lanes_ms": round(best["partial_lanes"], 3),
                      "matches": len(out), "same_as_order0": bool(same)}
        print(order, res[order], flush=True)
    print(json.dumps({"rows": n, "keys": keys, "query": Q, "by_order_path": res}))


if __name__ == "__main__":
    main()
