"""Vectorised numpy restatement of the absence closed form -- TEST INFRASTRUCTURE ONLY.

The CPU oracle (oracle/oracle.cpp) walks the reference's pending lists and timer FIFO literally and runs at
a few thousand events/s on C4, so it checks the HIP path at small sizes; this restatement is pinned against
the oracle (tests/test_absent_closed_form.py) and then checks the HIP path at the full C4 size (10M events).

Query shape: every e1=S -> not S[id==e1.id] for W (one stream, @app:playback, unpartitioned), rows in
arrival order with non-decreasing ts; `sel` = the e1 attributes the select projects.
    partial i is killed iff the next row j > i with id_j == id_i has ts_j < ts_i + W
    otherwise emitted before the first row with ts >= ts_i + W (trigger), ts = ts_i + W,
    callback group = rank among the emissions of that trigger.
"""
import numpy as np


def absent_every_eq(ts, ids, W, sel, base_index=0, stream=None):
    """stream: optional per-row stream index; rows of other streams (!= 0) only advance the clock."""
    n = len(ts)
    rows = np.arange(n) if stream is None else np.nonzero(stream == 0)[0]
    order = rows[np.argsort(ids[rows], kind="stable")]
    sid = ids[order]
    nxt = np.full(n, -1, np.int64)
    if len(order) > 1:
        same = sid[1:] == sid[:-1]
        nxt[order[:-1][same]] = order[1:][same]
    dl = ts + W
    killed = (nxt >= 0) & (ts[np.maximum(nxt, 0)] < dl)
    trig = np.searchsorted(ts, dl, side="left")
    emit = np.zeros(n, bool)
    emit[rows] = True
    emit &= ~killed & (trig < n)
    e = np.nonzero(emit)[0]
    t = trig[e]
    first = np.searchsorted(t, t, side="left")
    group = (np.arange(len(e)) - first).astype(np.uint32)
    vals = np.stack([c[e].astype(np.int64) for c in sel], axis=1) if sel else np.zeros((len(e), 0), np.int64)
    return dict(trigger=(t + base_index).astype(np.uint64), ts=dl[e], group=group, vals=vals)
