"""The headline pinned exactly as bench.py runs it (VERDICT r05 "next" 2).

bench.py's `value` is BASELINE configs[4]: the 1B-event, 1M-key C5 stream generated in HBM
(router.shard_stream_torch, one rank), pushed through `sg_push` in 500M-row batches with every key's partial
matches carried between them.  This test runs that same path -- same generator, same key ids, same global event
indices, same push size -- and compares every delivered row of every push with the oracle run key-sharded over the
host cores whose engines, and so their per-key pending lists, persist across the same pushes
(parity_util.CarriedShardedOracle).  Keys never interact (each has its own cloned runtime,
C/partition/PartitionRuntime.java:255-308) and a key's pending list is StreamPreStateProcessor's
(C/query/input/stream/state/StreamPreStateProcessor.java:292-337), so the stable merge by trigger of the shards'
outputs is the reference's delivery order for the whole push.

SG_C5_WHOLE=1 runs the whole stream (two 500M-row pushes, ~399M matches, several minutes); the default runs the
first 60M events of the same stream as two 30M-row pushes through the same code."""
import os
import threading
import time

import numpy as np
import pytest

from parity_util import CarriedShardedOracle, assert_same
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, Outputs

pytestmark = pytest.mark.gpu


def _heartbeat(stop, t0):
    while not stop.wait(30):
        print(f"  ... {time.time() - t0:.0f} s", flush=True)


@pytest.mark.timeout(1150)
def test_c5_headline_pushes_against_carried_oracle():
    import torch
    from siddhi_amd import _native as N
    from siddhi_amd import compiler as C
    from siddhi_amd import lowering as L
    from siddhi_amd import router
    whole = os.environ.get("SG_C5_WHOLE") == "1"
    _, n_total, K, R = synth.CONFIGS["C5"]
    total = n_total if whole else 60_000_000
    push_rows = 500_000_000 if whole else 30_000_000
    dev = torch.device("cuda", 0)
    cat, key_bound, _ = router.shard_stream_torch("C5", 0, 1, total, K, R, dev)
    q = synth.QUERIES["C5"]
    app = C.parse(q)
    p = app.partitions[0]
    nfa = L.lower(L.make_context(app, p.queries[0], p, {}))
    nsel = len(nfa.select)
    opts = N.sg_options()
    opts.no_carry = 0
    h = N.Handle(N.build_desc(nfa), device=0, options=opts)
    oracle = CarriedShardedOracle(q, max(2, min(16, os.cpu_count() or 2)))
    stop = threading.Event()
    t0 = time.time()
    threading.Thread(target=_heartbeat, args=(stop, t0), daemon=True).start()
    matches = 0
    try:
        for lo in range(0, total, push_rows):
            hi = min(total, lo + push_rows)
            keep = []
            cp = [cat["id"].data_ptr() + 8 * lo, cat["key"].data_ptr() + 4 * lo, cat["price"].data_ptr() + 4 * lo]
            b = N.make_batch(hi - lo, int(cat["gidx"][lo].item()), cat["ts"].data_ptr() + 8 * lo, 0,
                             cat["key"].data_ptr() + 4 * lo, cp, [0, 0, 0], 1, key_bound, keep,
                             index=cat["gidx"].data_ptr() + 8 * lo)
            h.push(b)
            torch.cuda.synchronize()
            tr, ts, ky, gr, vals, vn = h.poll(nsel)
            vnull = np.zeros((len(tr), nsel), np.uint8)
            for k in range(nsel):
                vnull[:, k] = (vn >> np.uint32(k)) & np.uint32(1)
            got = Outputs(tr, ts, ky, gr, vals, vnull)
            del tr, ts, ky, gr, vals, vn, vnull
            hb = Batch(hi - lo, 0, cat["ts"][lo:hi].cpu().numpy(), np.zeros(hi - lo, np.int32),
                       cat["key"][lo:hi].cpu().numpy(), [cat["id"][lo:hi].cpu().numpy(), cat["key"][lo:hi].cpu().numpy(),
                                                         cat["price"][lo:hi].cpu().numpy()], [None] * 3,
                       index=cat["gidx"][lo:hi].cpu().numpy().astype(np.uint64))
            want = oracle.push(hb)
            del hb
            assert len(got) == len(want) > 0, (lo, len(got), len(want))
            assert_same(got, want)
            matches += len(got)
            print(f"push [{lo}, {hi}): {len(got)} matches equal the carried oracle's ({time.time() - t0:.0f} s)",
                  flush=True)
            del got, want
    finally:
        stop.set()
        oracle.close()
        h.close()
    if whole:
        assert matches == 399_303_893   # bench.py's C5 count
