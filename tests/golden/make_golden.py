#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz): for each benchmark config, a small
synthetic input slice (SplitMix64 generator) and the ordered match output of the CPU oracle
(oracle/oracle.cpp, the C++ restatement of the reference state processors, itself pinned by the 18
reference KATs in tests/kats.py).  The reference (Java, unvendored jars) cannot be run in this image
(SURVEY.md §8c), so these are oracle outputs, frozen: they pin the oracle against drift and give the GPU
path fixed input/expected-output pairs that need no oracle at test time.

    python tests/golden/make_golden.py        # rewrites tests/golden/<case>.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# name: (config, events, keys (ids for C4), rate events/ms)
CASES = {
    "c1": ("C1", 40_000, 1, 1),
    "c2": ("C2", 40_000, 200, 20),
    "c3": ("C3", 60_000, 200, 100),
    "c3b": ("C3b", 40_000, 200, 100),
    "c3c": ("C3c", 40_000, 200, 20),
    "c4": ("C4", 8_000, 3_000, 1),
    "c5": ("C5", 60_000, 5_000, 200),
    # select arithmetic + having (QuerySelector over the math executors)
    "c2_sel": ("C2", 40_000, 200, 20),
    "c3b_sel": ("C3b", 40_000, 200, 100),
    "c4_sel": ("C4", 8_000, 3_000, 1),
}

# query text per case (default: the config's query, siddhi_amd/synth.py)
SELECT_QUERIES = {
    "c2_sel": ("define stream StockStream (id long, symbol string, price float); "
               "partition with (symbol of StockStream) begin @info(name='q') "
               "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
               "select e1.id as id1, e2.id - e1.id as gap, e2.price - e1.price as dp, e2.price / e1.price as ratio, "
               "(e2.price * 100) % 7 as m having dp > 5.0 or m < 1 insert into M; end;"),
    "c3b_sel": ("define stream S (id long, symbol string, v int, w int); "
                "partition with (symbol of S) begin @info(name='q') "
                "from every e1=S[v>500], e2=S[v>e1.v]<1:5>, e3=S[v<e1.v] or e4=S[w<e1.w] "
                "select e1.id as i1, e2[last].id - e2[0].id as span, e3.id + 1 as i3p, e4.id * 2 as i4d, "
                "e2[last].v - e1.v as dv, e1.w / (e1.v - 500) as q having i3p is null and span > 0 "
                "insert into M; end;"),
    "c4_sel": ("@app:playback define stream S (id long, seq long); define stream Tick (x int); "
               "@info(name='q') from every e1=S -> not S[id==e1.id] for 5 sec "
               "select e1.seq * 10 + e1.id as k, e1.id % 7 as m, e1.seq / 3 as t having m == 3 insert into M;"),
}


def query_of(name):
    from siddhi_amd import synth
    return SELECT_QUERIES.get(name) or synth.QUERIES[CASES[name][0]]


def golden_batch(cfg, n, keys, rate):
    """The fixture's input batch (C4 gets the closing Tick event that fires the remaining timers)."""
    from parity_util import dense_first_seen, synth_batch
    from siddhi_amd.runtime import Batch
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    if cfg.startswith("C4"):
        ts = np.append(b.ts, b.ts[-1] + 5001)
        st = np.append(b.stream, np.int32(1)).astype(np.int32)
        cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
        return Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)
    b.key = dense_first_seen(b.key)
    return b


def save(name, cfg, b, out):
    arrs = {"cfg": np.array(cfg), "ts": b.ts, "stream": b.stream, "key": b.key,
            "ncols": np.array(len(b.cols))}
    for i, c in enumerate(b.cols):
        arrs[f"col{i}"] = c
    for f in ("trigger", "ts", "key", "group", "vals", "vnull"):
        arrs["out_" + f] = getattr(out, f)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)


def load(name):
    """(query text, Batch, expected Outputs) of one fixture."""
    from siddhi_amd import synth
    from siddhi_amd.runtime import Batch, Outputs
    z = np.load(os.path.join(HERE, name + ".npz"))
    cfg = str(z["cfg"])
    cols = [z[f"col{i}"] for i in range(int(z["ncols"]))]
    n = len(z["ts"])
    b = Batch(n, 0, z["ts"], z["stream"], z["key"], cols, [None] * len(cols))
    want = Outputs(*[z["out_" + f] for f in ("trigger", "ts", "key", "group", "vals", "vnull")])
    return query_of(name), b, want


def main(only=None):
    from oracle import OracleEngine
    from parity_util import run_engine
    from siddhi_amd import synth
    for name, (cfg, n, keys, rate) in CASES.items():
        b = golden_batch(cfg, n, keys, rate)
        if only and name not in only:
            continue
        out = run_engine(OracleEngine, query_of(name), [b])
        save(name, cfg, b, out)
        print(f"{name}: {cfg} {n} events -> {len(out)} matches")


if __name__ == "__main__":
    main(set(sys.argv[1:]) or None)    # optional case names: regenerate only those
