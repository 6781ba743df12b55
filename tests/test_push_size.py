"""The headline's push size is an ingress choice, not a semantic one.

bench.py pushes BASELINE configs[4]'s 1B-event C5 stream in batches of `--c5-push-rows` with per-key state carried
between pushes.  test_node.py::test_node_c5_whole_1b_stream_ten_pushes pins 100M-row pushes to the carried,
key-sharded oracle row for row; this test shows that other push sizes produce byte-identical match records in the
same global order, so every push size the bench uses inherits that pin.  The records are compared through an
order-sensitive checksum computed on the GPU over every 64-bit word of every record (word value x position), with
the match count; the reference has no push at all (StreamJunction hands events over one by one,
`C/stream/StreamJunction.java`), so its output cannot depend on the batching.
"""
import ctypes as ct
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
GOLD = 0x9E3779B97F4A7C15 - (1 << 64)   # (as a signed 64-bit value)


def _stream_digest(cat, key_bound, push_rows):
    """(matches, checksum) of the C5 stream in `cat` pushed in batches of push_rows (state carried)."""
    import torch
    from siddhi_amd import _native as N
    from siddhi_amd import compiler as C
    from siddhi_amd import lowering as L
    from siddhi_amd import synth
    app = C.parse(synth.QUERIES["C5"])
    p = app.partitions[0]
    nfa = L.lower(L.make_context(app, p.queries[0], p, {}))
    opts = N.sg_options()
    opts.no_carry = 0
    h = N.Handle(N.build_desc(nfa), device=torch.cuda.current_device(), options=opts)
    hip = ct.CDLL("libamdhip64.so")
    stream = torch.cuda.current_stream()
    h.check(h.lib.sg_set_stream(h.h, stream.cuda_stream))
    n = cat["ts"].numel()
    keep = []
    total, acc = 0, torch.zeros((), dtype=torch.int64, device="cuda")
    for lo in range(0, n, push_rows):
        hi = min(n, lo + push_rows)
        cp = [cat["id"].data_ptr() + 8 * lo, cat["key"].data_ptr() + 4 * lo, cat["price"].data_ptr() + 4 * lo]
        b = N.make_batch(hi - lo, int(cat["gidx"][lo].item()), cat["ts"].data_ptr() + 8 * lo, 0,
                         cat["key"].data_ptr() + 4 * lo, cp, [0, 0, 0], 1, key_bound, keep,
                         index=cat["gidx"].data_ptr() + 8 * lo)
        h.push(b)
        m = h.device_records()
        if m.n:
            assert m.record_bytes % 8 == 0
            words = m.record_bytes // 8
            torch.cuda.synchronize()
            for s0 in range(0, m.n, 1 << 25):   # 32M records (2 GB) at a time
                k = min(m.n - s0, 1 << 25)
                buf = torch.empty((k, words), dtype=torch.int64, device="cuda")
                assert hip.hipMemcpy(ct.c_void_p(buf.data_ptr()), ct.c_void_p(m.base + s0 * m.record_bytes),
                                     ct.c_size_t(k * m.record_bytes), 3) == 0   # hipMemcpyDeviceToDevice
                pos = torch.arange(total + s0, total + s0 + k, dtype=torch.int64, device="cuda").unsqueeze(1) * words
                pos = pos + torch.arange(words, dtype=torch.int64, device="cuda")
                acc += ((buf ^ (pos * GOLD)) * (pos | 1)).sum()   # int64 arithmetic wraps
                del buf, pos
        total += m.n
        h.check(h.lib.sg_discard(h.h))   # (records accumulate until delivered)
    torch.cuda.synchronize()
    h.close()
    return total, int(acc.item())


def test_c5_stream_push_size_does_not_change_records():
    import torch
    from siddhi_amd import router, synth
    _, n_total, keys, rate = synth.CONFIGS["C5"]
    cat, key_bound, _ = router.shard_stream_torch("C5", 0, 1, n_total, keys, rate, torch.device("cuda", 0))
    base = _stream_digest(cat, key_bound, 100_000_000)
    assert base[0] == 399_303_893   # the ten-push oracle run's count (profiles/r04/c5_whole_1b_test_final.log)
    for rows in (500_000_000, 1_000_000_000):
        assert _stream_digest(cat, key_bound, rows) == base, rows
