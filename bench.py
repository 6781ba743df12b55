#!/usr/bin/env python3
"""Benchmark: events/sec of the partitioned pattern query on MI355X (BASELINE.json metric; its config, configs[4] = C5).

Headline workload:
  partition with (symbol of StockStream) begin
    from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
    select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;
  ONE 1B-event stream over 1M keys at 10,000 events/ms (SplitMix64 generator, siddhi_amd/synth.py).

value (task contract: inputs already resident in HBM when the timed region starts): the stream is split by key hash
  across the N ranks (router.shard_of_torch: mix64(key) mod N, computed on the GPU; strong scaling -- the same stream
  at every N, no data-path collective: keys never interact); each rank pushes its share in 500M-row
  batches (tests/test_push_size.py: records identical to 100M-row pushes) with per-key state carried between them, every match projected in HBM (sg_device_records, zero-copy).
  A step = the whole stream; value = 1e9 events / max-over-ranks step time.
whole_node (SURVEY.md §8d's definition, never `value`): pinned raw host rows (64-bit symbol values) -> sg_node_push
  (native router, per-GPU chunked H2D / kernels / D2H, native merge) -> every match tuple in host memory; with the
  PCIe rate against a measured pinned-copy peak, and on one GPU the host stages of G = 2, 4, 8 shards mapped onto it.
configs: C2 (configs[1]), C1, C3b, C3c, C4 and PP sub-lines, one push each on one GPU, with their own rooflines.

roofline (per launch = per push): SURVEY §8d's algorithmic bytes of the push over the dominant kernel's average
duration (largest HIP-event time, recorded on the launch stream by the engine, sg_timing.kernel_ms) -- the task's
definition -- with beside it the same kernel against ITS OWN algorithmic bytes (`kernel_own`, KERNEL_BYTES), the §8d
bytes over the sum of the push's kernels (`path`), and the predicate pass (4.125 B/event); `traffic` comes from a
rocprofv3 PMC summary of this same command (profiles/r05/collect.sh, FETCH_SIZE x2 + WRITE_SIZE passes) and is only
used when its kernel-source hash matches the tree.
The JSON line ends with `whole_node` and `roofline` (the driver keeps the line's tail).
"""
import argparse
import hashlib
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from siddhi_amd import _native as N          # noqa: E402
from siddhi_amd import compiler as C          # noqa: E402
from siddhi_amd import lowering as L          # noqa: E402
from siddhi_amd import synth                  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
PMC_DIR = os.path.join(ROOT, "profiles", "r06")


def barrier():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()


def reduce_max(x):
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x):
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM)
    return float(t.item())


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


# sources of the engine routes that do not run the closed-form walker (C1/C2/C5): their edits leave a C2 profile valid
NODE_ONLY = ("node.hip", "keydict.hip", "keydict.h", "router.cpp")
OTHER_ROUTES = ("absent.hip", "interp.hip", "interp.h", "partial.hip", "chain.h", "seq.h", "router.cpp")


def source_hash(cfg="C2"):
    """Hash of everything the measured kernels are built from (a PMC summary is valid only for this tree): for the
    closed-form configs the sources of the other routes are left out."""
    h = hashlib.sha256()
    files = []
    for d, exts in ((os.path.join(ROOT, "siddhi_amd", "csrc"), (".hip", ".h", ".cpp")),
                    (os.path.join(ROOT, "include"), (".h",))):
        files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))
    files = [f for f in files if os.path.basename(f) not in NODE_ONLY]   # not on the per-push path measured here
    if cfg in ("C1", "C2", "C5"):
        files = [f for f in files if os.path.basename(f) not in OTHER_ROUTES]
    files.append(os.path.join(ROOT, "siddhi_amd", "lowering.py"))
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def make_handle(cfg, no_carry=1, ingress_rows=0):
    app = C.parse(synth.QUERIES[cfg])
    if app.partitions:
        p = app.partitions[0]
        ctx = L.make_context(app, p.queries[0], p, {})
    else:
        ctx = L.make_context(app, app.queries[0], None, {})
    nfa = L.lower(ctx)
    opts = N.sg_options()
    opts.no_carry = no_carry
    opts.ingress_rows = ingress_rows
    return N.Handle(N.build_desc(nfa), device=torch.cuda.current_device(), options=opts), nfa


def _oracle_paths():
    for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


def host_info():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except Exception:
        nproc = os.cpu_count()
    return {"nproc": nproc, "cpu_model": model}


def cpu_baseline(cfg, n_sample, keys, rate):
    """Oracle (C++ restatement of the reference state processors), 1 thread, first n_sample rows: the
    reference's synchronous single-thread InputHandler.send path."""
    _oracle_paths()
    from oracle import OracleEngine
    from parity_util import run_engine, synth_batch
    b = synth_batch(cfg, 0, n_sample, keys=keys, rate=rate)
    t0 = time.perf_counter()
    out = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    dt = time.perf_counter() - t0
    return n_sample / dt, len(out), dt


_MC = {}


def _mc_worker(w):
    from oracle import OracleEngine
    from parity_util import run_engine
    b = _MC["shards"][w]
    t0 = time.perf_counter()
    out = run_engine(OracleEngine, synth.QUERIES[_MC["cfg"]], [b])
    return time.perf_counter() - t0, len(out)


def cpu_baseline_multicore(cfg, n_sample, keys, rate, workers):
    """The same oracle on the host cores the box grants this job: rows sharded by partition key across worker
    processes (keys never interact), each shard keeping its global event indices."""
    import multiprocessing as mp
    _oracle_paths()
    from parity_util import synth_batch
    from siddhi_amd.runtime import Batch
    b = synth_batch(cfg, 0, n_sample, keys=keys, rate=rate)
    shards = []
    for w in range(workers):
        ix = np.nonzero((b.key % workers) == w)[0]
        shards.append(Batch(len(ix), 0, b.ts[ix], b.stream[ix], b.key[ix], [c[ix] for c in b.cols],
                            [None] * len(b.cols), index=ix.astype(np.uint64)))
    _MC["shards"], _MC["cfg"] = shards, cfg
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        t0 = time.perf_counter()
        res = pool.map(_mc_worker, range(workers))
        dt = time.perf_counter() - t0
    return n_sample / dt, sum(r[1] for r in res), dt


def pmc_traffic(path, cfg, n, dominant):
    """HBM-side bytes per launch of the dominant kernel and per push of the whole path, from a committed
    rocprofv3 PMC summary of this command -- only if it was collected on this exact kernel source."""
    try:
        with open(path) as f:
            prof = json.load(f)
    except OSError:
        return None, "no PMC summary at %s" % os.path.relpath(path, ROOT)
    if prof.get("source_hash") != source_hash(cfg):
        return None, "stale PMC summary (source hash %s != tree %s): rerun profiles/r05/collect.sh" % (
            prof.get("source_hash"), source_hash(cfg))
    if prof.get("workload") != cfg or prof.get("events") != n:
        return None, "PMC summary is for %s/%s events" % (prof.get("workload"), prof.get("events"))
    k = prof["kernels"].get(dominant)
    dom = None if k is None else round(k["bytes_per_push"] / 1e9, 4)
    # runtime fills / copies (hipMemset, the output buffer's growth in the warm-up step) are averaged over every
    # push of the profiled run: reported beside the kernels' bytes, not in them
    rt = prof["kernels"].get("runtime_fill_copy", {}).get("bytes_per_push", 0.0)
    path_tot = sum(v["bytes_per_push"] for m, v in prof["kernels"].items() if m != "runtime_fill_copy")
    return {"dominant_GB": dom, "path_GB": round(path_tot / 1e9, 4), "runtime_fill_copy_GB": round(rt / 1e9, 4),
            "source": os.path.relpath(path, ROOT), "collected_at_head": prof.get("git_head")}, None


def attach_traffic(roof, path, cfg, n):
    tr, why = pmc_traffic(path, cfg, n, roof["kernel"])
    if tr is not None:
        roof["traffic"] = tr["dominant_GB"]
        roof["traffic_unit"] = "GB per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM)"
        roof["path_traffic_GB"] = tr["path_GB"]
        roof["runtime_fill_copy_GB"] = tr["runtime_fill_copy_GB"]
        roof["traffic_source"] = tr["source"]
    else:
        roof["traffic_note"] = why
    return roof


def synth_columns(cfg, rank, n, keys, rate, dev):
    g = synth.generate_torch(cfg, rank * n, n, dev, keys=keys, rate=rate)
    key = g["key"].to(torch.int32) if "key" in g else torch.zeros(n, dtype=torch.int32, device=dev)
    if cfg.startswith("C4"):     # S(id, seq) rows only (the Tick stream's column is never read)
        cols = [g["id"], g["seq"], torch.zeros(n, dtype=torch.int32, device=dev)]
    elif cfg.startswith("PP"):   # Stream1 / Stream2 (symbol, price, volume)
        cols = [key, g["price"], key] * 2
    elif cfg.startswith("C3"):
        cols = [g["id"], key, g["v"], g["w"]]
    else:
        cols = [g["id"], key, g["price"]]
    return g, key, cols


def host_stream(cfg, total, keys, rate, dev, gen_rows=50_000_000):
    """The config's stream as the host receives it, in pinned memory: ts, the raw 64-bit partition-key value per
    row (synth.raw_symbols, never a dense id) and the query's typed columns.  Generated in HBM chunk by chunk and
    copied down (outside any timed region)."""
    keep = []

    def pinned(n, dt):
        p = N.PinnedArray(n, dt)
        keep.append(p)
        return p.array
    ts = pinned(total, np.int64)
    raw = pinned(total, np.int64)
    if cfg.startswith("C3"):
        names = [("id", np.int64), (None, np.int32), ("v", np.int32), ("w", np.int32)]
    else:
        names = [("id", np.int64), (None, np.int32), ("price", np.float32)]
    cols = [pinned(total, dt) if nm else None for nm, dt in names]
    for lo in range(0, total, gen_rows):
        hi = min(total, lo + gen_rows)
        g = synth.generate_torch(cfg, lo, hi - lo, dev, keys=keys, rate=rate)
        ts[lo:hi] = g["ts"].cpu().numpy()
        raw[lo:hi] = synth.raw_symbols_torch(g["key"]).cpu().numpy()
        for (nm, _), c in zip(names, cols):
            if nm:
                c[lo:hi] = g[nm].cpu().numpy()
        del g
    torch.cuda.empty_cache()
    return ts, raw, cols, keep


def node_whole(cfg, total, keys, rate, devices, steps, threads, chunk_rows, key_dict=0):
    """SURVEY.md §8d whole-node events/s through the node pipeline (sg_node_*, csrc/node.hip), one host process
    driving `gpus` GPUs: pinned raw host rows -> native router (first-seen dense ids, shard mix64(id) mod G) ->
    per-GPU threads (chunked H2D, kernels, GPU-transposed SoA match columns D2H, overlapped across chunks) ->
    native k-way merge into the node's delivery order -> every match tuple (trigger, ts, projected columns) in
    pinned host memory.  Routing and merge are inside the timed region; data generation is not."""
    gpus = len(devices)
    ts, raw, cols, keep = host_stream(cfg, total, keys, rate, torch.device("cuda", devices[0]))
    nfa = L.lower(_ctx(cfg))
    node = N.Node(N.build_desc(nfa), n_gpus=gpus, devices=list(devices), threads=threads, chunk_rows=chunk_rows)
    nb = N.make_node_batch(total, 0, ts.ctypes.data, 0, raw.ctypes.data, [c.ctypes.data if c is not None else 0
                                                                         for c in cols], [0] * len(cols), keep)
    cap = total // 2 + 1_000_000
    sink = N.ColumnSink(nfa, cap, pinned=True, fields=("trigger", "ts"), nulls=False)
    times, stats, got = [], [], 0
    for s in range(steps + 1):
        node.reset()
        if key_dict:
            node.set_key_dict(key_dict)
        t0 = time.perf_counter()
        got = node.push(nb, sink.struct, cap)
        dt = time.perf_counter() - t0
        if s:   # the first push sizes the pinned staging and device slots
            times.append(dt)
            stats.append(node.stats())
    # spot check of the delivered order: triggers never decrease
    tr = sink.trigger[:got]
    ordered = bool(np.all(tr[1:] >= tr[:-1])) if got > 1 else True
    node.close()
    ms = 1000.0 * float(np.mean(times))
    st = stats[-1]
    del sink, keep, ts, raw, cols
    return {"workload": f"{cfg}: " + synth.QUERIES[cfg], "events": total, "keys": keys,
            "rate_events_per_ms": rate, "gpus": gpus, "ms_per_step": round(ms, 2),
            "value": round(total / (ms * 1e-3), 1), "unit": "events/s", "matches": int(got),
            "delivery_ordered": ordered, "host_threads": threads, "chunk_rows": int(st["chunk_rows"]),
            "chunks": int(st["chunks"]), "route_ms": round(st["route_ms"], 1), "merge_ms": round(st["merge_ms"], 1),
            "gpu_busy_ms": [round(x, 1) for x in st["gpu_ms"][:gpus]],
            "h2d_GB": round(st["h2d_bytes"] / 1e9, 3), "d2h_GB": round(st["d2h_bytes"] / 1e9, 3),
            "shard_rows": [int(x) for x in st["shard_rows"][:gpus]],
            "definition": "SURVEY.md §8d: pinned raw host rows -> native router -> per-GPU chunked H2D / kernels / "
                          "D2H -> native merge -> every match tuple in host memory (sg_node_push wall time)"}


def _ctx(cfg):
    app = C.parse(synth.QUERIES[cfg])
    if app.partitions:
        p = app.partitions[0]
        return L.make_context(app, p.queries[0], p, {})
    return L.make_context(app, app.queries[0], None, {})


# SURVEY.md §8d algorithmic bytes per config: (whole path B/event, B/match, predicate pass B/event)
#   C1: ts 8 + price 4 + bit; C2/C5: + key 4; 36 B/match (trigger 8, rank 4, ts 8, two slot indices 8+8)
#   C3b/C3c: ts 8 + key 4 + v 4 + w 4 + bits; 92 B/match (trigger, rank, ts, 4 slots x 8, 5 projected x 8); the
#            predicate pass reads only v (e1's filter is the one event-local filter): 4.125 B/event, as its PMC
#            FETCH+WRITE shows (profiles/r03/C3b_pmc.json: 412.6 MB per 100M events)
#   C4: ts 8 + id 8 (no local predicate: no predicate pass); 28 B per emission (one slot)
PATH_BYTES = {"C1": (12.125, 36.0, 4.125), "C2": (16.125, 36.0, 4.125), "C5": (16.125, 36.0, 4.125),
              "PP": (20.125, 36.0, 4.125), "PPe": (20.125, 36.0, 4.125),   # + the stream column (4 B)
              "C3b": (20.125, 92.0, 4.125), "C3c": (20.125, 92.0, 4.125), "C3": (20.125, 92.0, 4.125),
              "C4": (16.0, 28.0, None)}

# Each kernel's OWN algorithmic bytes (B/event, B/match) on the closed-form path of C2/C5 (16-B walker records
# {dts, row|flags, price, id}; match records of 64 B = 32-B header + 4 projected values; e1's compact record 16 B):
#   pred         price 4 read + condition bit 0.125 written
#   part_hist    key 4 read
#   part_group   ts 8 + key 4 + price 4 + id 8 + bit 0.125 read; record 16 + in-group key 1 written
#   part_split   record 16 + supergroup key 2 read, record 16 + in-group key 1 written
#   gw_count     in-group key 1 read
#   group_walk   record 16 + in-group key 1 read; per match 8 B entry + per trigger (~1.3 matches) 16 B header and an
#                8 B trigger word written: ~26 B per match
#   gw_tiles     trigger word 8 read
#   gw_project   trigger word 8 read; per match its 8 B entry + the trigger's 16 B header (~12 per match) read, 64 B
#                record written
#   (sorted-walker pipeline: fewer than 65,536 keys (C2), or a push the group walker declines)
#   part_key     record 16 + key 1 read, record 16 written;  units/tile_transpose  record 16 read + 16 written
#   walk_count   record 16 read, count 4 written per match;   walk_record  record 16 read, 16 B per match written
#   project      16 B intermediate + 24 B trigger row read, 64 B record written per match
#   key_sort     rocPRIM onesweep over 16-B records + 4-B keys, 3 passes (C5's 1M keys), read + write
KERNEL_BYTES = {"pred": (4.125, 0.0), "part_hist": (4.0, 0.0), "part_group": (41.125, 0.0),
                "group_walk": (17.0, 26.0), "gw_project": (8.0, 84.0), "gw_tiles": (8.0, 0.0), "gw_count": (1.0, 0.0),
                "part_key": (33.0, 0.0),
                "tile_transpose": (32.0, 0.0), "walk_count": (16.0, 4.0), "walk_record": (16.0, 16.0),
                "project": (0.0, 104.0), "key_sort": (40.0, 0.0), "pack": (44.125, 0.0), "part_split": (35.0, 0.0),
                "nge_search": (12.125, 8.0), "once_match": (16.125, 0.0)}


def roofline_of(cfg, n, matches, kern, stage):
    """`roofline` of one push: SURVEY.md §8d bytes over the dominant kernel's HIP-event time (`achieved`, `frac`);
    `kernel_own` = the same kernel against its OWN algorithmic bytes (KERNEL_BYTES); `path` = §8d bytes over the sum
    of the push's kernels; the predicate-evaluation pass."""
    per_ev, per_m, pred_b = PATH_BYTES[cfg]
    path_bytes = per_ev * n + per_m * matches
    dominant = max(kern, key=kern.get) if kern else None
    t_dom = kern.get(dominant, 0.0)
    if dominant in KERNEL_BYTES:
        ke, km = KERNEL_BYTES[dominant]
        dom_bytes = ke * n + km * matches
        dom_def = "%s's own algorithmic bytes: %.3f B/event + %.0f B/match (bench.py KERNEL_BYTES)" % (dominant, ke, km)
    else:   # (lane / machine kernels: their bytes are the path's)
        dom_bytes = path_bytes
        dom_def = "SURVEY.md §8d whole-path bytes (%.3f B/event + %.0f B/match): no per-kernel model" % (per_ev, per_m)
    dom_gbs = dom_bytes / (t_dom * 1e-3) / 1e9 if t_dom else 0.0
    s8_gbs = path_bytes / (t_dom * 1e-3) / 1e9 if t_dom else 0.0
    path_gbs = path_bytes / (stage[4] * 1e-3) / 1e9 if stage[4] else 0.0
    roof = {"bound": "hbm", "achieved": round(s8_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(s8_gbs / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": dominant, "kernel_ms": round(t_dom, 4),
            "algorithmic_GB_per_launch": round(path_bytes / 1e9, 4),
            "bytes_definition": "SURVEY.md §8d: %.3f B/event + %.0f B/match over the dominant kernel's time" % (per_ev, per_m),
            "kernel_own": {"achieved": round(dom_gbs, 1), "frac": round(dom_gbs / HBM_PEAK_GBS, 4),
                           "algorithmic_GB": round(dom_bytes / 1e9, 4), "bytes_definition": dom_def},
            "path": {"achieved": round(path_gbs, 1), "frac": round(path_gbs / HBM_PEAK_GBS, 4),
                     "kernels_total_ms": round(float(stage[4]), 4), "algorithmic_GB": round(path_bytes / 1e9, 4),
                     "bytes_definition": "SURVEY.md §8d: %.3f B/event + %.0f B/match" % (per_ev, per_m)},
            "kernels_ms": {k: round(v, 4) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])}}
    if "pred" in kern and pred_b:
        pg = pred_b * n / (kern["pred"] * 1e-3) / 1e9
        roof["pred_eval_pass"] = {"achieved": round(pg, 1), "frac": round(pg / HBM_PEAK_GBS, 4),
                                  "bytes_per_event": pred_b, "ms": round(kern["pred"], 4)}
    return roof


def measure_push(cfg, rank, n, keys, rate, dev, steps, warmup, sync_ranks=False):
    """K timed sg_push steps of one batch resident in HBM (fresh state each step), HIP-event kernel times."""
    g, key, cols = synth_columns(cfg, rank, n, keys, rate, dev)
    torch.cuda.synchronize()
    keep = []
    h, nfa = make_handle(cfg)   # each step is a complete stream: no state carried between steps
    partitioned = "partition with" in synth.QUERIES[cfg]
    batch = N.make_batch(n, rank * n, g["ts"].data_ptr(), g["stream"].data_ptr() if "stream" in g else 0, key.data_ptr(),
                         [c.data_ptr() for c in cols], [0] * len(cols), 1, keys if partitioned else 1, keep)
    stream = torch.cuda.current_stream()
    h.check(h.lib.sg_set_stream(h.h, stream.cuda_stream))
    tick = int(synth.T0 + (n - 1) // rate + 5001)   # C4: the final Tick fires every remaining timer
    timings = []

    def step(record=False):
        h.reset()
        h.push(batch)
        if record:
            timings.append(h.timing())
        if cfg.startswith("C4"):
            h.advance_time(tick, rank * n + n)
            if record:
                timings.append(h.timing())
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if sync_ranks:
        barrier()
    torch.cuda.synchronize()
    stage = np.zeros(5)
    kern = {}
    matches = spilled = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        timings.clear()
        step(record=True)
        for t in timings:   # (C4: the push and the final clock advance)
            stage += [t.pred_ms, t.partition_ms, t.match_ms, t.output_ms, t.total_ms]
            for name, ms in t.kernels():
                kern[name] = kern.get(name, 0.0) + ms
        matches = h.pending() if cfg.startswith("C4") else timings[0].matches
        spilled = timings[0].spilled_units
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if sync_ranks:
        elapsed = reduce_max(elapsed)
        barrier()
    h.close()
    del g, key, cols
    torch.cuda.empty_cache()
    return {"elapsed": elapsed, "stage": stage / steps, "kern": {k: v / steps for k, v in kern.items()},
            "matches": matches, "spilled": spilled}


def stream_line(cfg, dev, steps, warmup, pushes=2, lateness=-1):
    """A config as a stream (VERDICT r05 "next" 6): its 100M events pushed in `pushes` consecutive batches with every
    key's pending partials carried between them (no_carry = 0) -- the streaming cost, which for count-waiting partial
    lanes includes walking to the key's end (a count state never expires a partial, CountPreStateProcessor.java:53-93).
    lateness >= 0 sets sg_options.bounded_lateness (the caller's bound on rows arriving behind the clock; the synthetic
    stream is monotone), under which such a partial stops at `within` + lateness of e1."""
    _, n_cfg, keys, rate = synth.CONFIGS[synth._base(cfg)]
    n = min(n_cfg, 100_000_000)
    g, key, cols = synth_columns(cfg, 0, n, keys, rate, dev)
    torch.cuda.synchronize()
    h, nfa = make_handle(cfg, no_carry=0)
    if lateness >= 0:
        h.opts.bounded_lateness = 1
        h.opts.max_lateness_ms = lateness
        h.close()
        h = N.Handle(h.desc, device=torch.cuda.current_device(), options=h.opts)
    keep, batches = [], []
    per = (n + pushes - 1) // pushes
    for lo in range(0, n, per):
        hi = min(n, lo + per)
        batches.append(N.make_batch(hi - lo, lo, g["ts"].data_ptr() + 8 * lo, 0, key.data_ptr() + 4 * lo,
                                    [c.data_ptr() + c.element_size() * lo for c in cols], [0] * len(cols), 1, keys, keep))
    h.check(h.lib.sg_set_stream(h.h, torch.cuda.current_stream().cuda_stream))
    kern, matches = {}, 0

    def step(record=False):
        nonlocal matches
        h.reset()
        matches = 0
        for b in batches:
            h.push(b)
            t = h.timing()
            matches += t.matches
            if record:
                for name, ms in t.kernels():
                    kern[name] = kern.get(name, 0.0) + ms
            h.discard()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(record=True)
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - t0) / steps
    h.close()
    del g, key, cols, batches
    torch.cuda.empty_cache()
    return {"workload": f"{cfg} as a stream of {pushes} pushes, state carried" +
                        (f", bounded lateness {lateness} ms" if lateness >= 0 else ""),
            "events": n, "pushes": pushes, "matches": int(matches), "steps": steps, "ms_per_stream": round(ms, 3),
            "value": round(n / (ms * 1e-3), 1), "unit": "events/s",
            "kernels_ms_per_stream": {k: round(v / steps, 3) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])[:8]}}


CPU_SAMPLE = {"PP": 12_000_000, "PPe": 12_000_000, "C1": 1_000_000, "C2": 12_000_000, "C3b": 6_000_000, "C3c": 3_000_000, "C4": 60_000, "C5": 3_000_000}


def config_line(cfg, dev, steps, warmup, cpu):
    """One BASELINE config beside the headline: its own push timing, roofline with its own §8d bytes, and the
    oracle on a bounded sample of the same stream (1 thread)."""
    _, n_cfg, keys, rate = synth.CONFIGS[synth._base(cfg)]
    n = min(n_cfg, 100_000_000)
    m = measure_push(cfg, 0, n, keys, rate, dev, steps, warmup)
    ms = 1000.0 * m["elapsed"] / steps
    out = {"workload": f"{cfg}: " + synth.QUERIES[cfg], "events": n, "keys": keys, "rate_events_per_ms": rate,
           "matches": int(m["matches"]), "steps": steps, "ms_per_push": round(ms, 3),
           "value": round(n / (ms * 1e-3), 1), "unit": "events/s",
           "roofline": attach_traffic(roofline_of(cfg, n, m["matches"], m["kern"], m["stage"]),
                                      os.path.join(PMC_DIR, cfg + "_pmc.json"), cfg, n)}
    if cpu:
        sample = CPU_SAMPLE[cfg] // 4
        r, nm, dt = cpu_baseline(cfg, sample, keys, rate)
        out["cpu_baseline"] = {"value": round(r, 1), "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": f"first {sample} events, oracle single thread, {nm} matches, {dt:.1f}s"}
    return out


def c5_stream(rank, ws, dev, steps, warmup, total, push_rows):
    """BASELINE configs[4] as it is worded: ONE 1B-event, 1M-key C5 stream sharded by key hash across the node's
    ranks (strong scaling: the stream is the same at every N).  Every rank generates the global stream in HBM chunk
    by chunk and keeps the rows of the keys it owns (siddhi_amd/router.py shard_of_torch: mix64(key) mod N, the host
    router's assignment, computed on the GPU), with its own dense key ids and the rows' global event indices; it then
    pushes its share as consecutive batches of `push_rows` (state carried between pushes).  Time = max over ranks;
    value = the whole stream's events / that time.  Merging the ranks' match streams (router.merge) is host work
    outside this number; tests/test_multigpu.py checks the merged output against the oracle.  Kernel times (HIP events
    on the launch stream, summed over a step's pushes) give the roofline of rank 0's share."""
    from siddhi_amd import router
    _, n_total, keys, rate = synth.CONFIGS["C5"]
    total = total or n_total
    cat, key_bound, _ = router.shard_stream_torch("C5", rank, ws, total, keys, rate, dev)
    n = cat["ts"].numel()
    h, nfa = make_handle("C5", no_carry=0)
    keep, batches = [], []
    for lo in range(0, n, push_rows):
        hi = min(n, lo + push_rows)
        cp = [cat["id"].data_ptr() + 8 * lo, cat["key"].data_ptr() + 4 * lo, cat["price"].data_ptr() + 4 * lo]
        # (one rank keeps every row: its rows' global indices are base_index + row, so the batch needs no index column;
        #  with N ranks each rank's rows are a subsequence and carry their global indices)
        batches.append(N.make_batch(hi - lo, int(cat["gidx"][lo].item()), cat["ts"].data_ptr() + 8 * lo, 0,
                                    cat["key"].data_ptr() + 4 * lo, cp, [0, 0, 0], 1, key_bound, keep,
                                    index=cat["gidx"].data_ptr() + 8 * lo if ws > 1 else 0))
    stream = torch.cuda.current_stream()
    h.check(h.lib.sg_set_stream(h.h, stream.cuda_stream))
    stage = np.zeros(5)
    kern = {}

    def step(record=False):
        h.reset()
        m = 0
        for b in batches:
            h.push(b)
            t = h.timing()
            m += t.matches
            if record:
                stage[:] += [t.pred_ms, t.partition_ms, t.match_ms, t.output_ms, t.total_ms]
                for name, ms in t.kernels():
                    kern[name] = kern.get(name, 0.0) + ms
        return m

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        matches = step(record=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el, all_matches, rows = reduce_max(el), reduce_sum(matches), reduce_sum(n)
    h.close()
    del cat, batches
    torch.cuda.empty_cache()
    ms = 1000.0 * el / steps
    # per launch (= per push): the step's kernel times and bytes over its pushes
    pushes = max(1, len(range(0, n, push_rows)))
    roof = roofline_of("C5", n / pushes, matches / pushes, {k: v / steps / pushes for k, v in kern.items()},
                       stage / steps / pushes)
    roof["scope"] = "per push (launch) of rank 0's share of the stream: %d events in %d pushes of <= %d rows, %d matches" % (
        n, pushes, push_rows, matches)
    roof["push_events"] = int(round(n / pushes))
    return {"workload": "C5 (BASELINE configs[4]): " + synth.QUERIES["C5"], "events": total, "keys": keys,
            "rate_events_per_ms": rate, "n_gpus": ws, "scaling": "strong", "steps": steps,
            "ms_per_step": round(ms, 3), "value": round(total / (ms * 1e-3), 1), "unit": "events/s",
            "matches": int(all_matches), "rows_routed": int(rows), "push_rows": push_rows,
            "sharding": "mix64(key) mod N on the GPU (router.shard_of_torch), per-rank dense ids, global indices kept",
            "data": "synthetic, generated in HBM; inputs resident before the timed region", "roofline": roof}


def pcie_peak(dev, mib=1024, reps=5):
    """Pinned host -> HBM copy rate of one large hipMemcpy on this box (the whole-node path's PCIe ceiling)."""
    src = torch.empty(mib << 20, dtype=torch.uint8).pin_memory()
    dst = torch.empty(mib << 20, dtype=torch.uint8, device=dev)
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    del src, dst
    return (mib << 20) / best / 1e9


TORCHRUN_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
                "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def whole_node_block(args, ws, local, dev):
    """SURVEY.md §8d whole-node rate: the 1B-event C5 stream from pinned host memory through sg_node_push"""
    c5w = None
    try:
        thr = args.node_threads or max(16, min(16 * ws, len(os.sched_getaffinity(0))))
        devs = [int(x) for x in args.c5_node_devices.split(",")] if args.c5_node_devices else list(range(ws))
        c5w = node_whole("C5", args.c5_events or synth.CONFIGS["C5"][1], synth.CONFIGS["C5"][2],
                         synth.CONFIGS["C5"][3], devs, args.c5_node_steps, thr, 0)
        pk = pcie_peak(dev)
        h2d_rate = c5w["h2d_GB"] / (c5w["ms_per_step"] * 1e-3)
        c5w["pcie"] = {"h2d_GBs": round(h2d_rate, 1), "peak_h2d_GBs": round(pk, 1),
                       "pcie_frac": round(h2d_rate / pk / max(1, len(devs)), 4),
                       "peak_definition": "one 1 GiB pinned -> HBM copy on this box (best of 5), per GPU"}
        shards = [int(x) for x in args.node_shards.split(",") if x] if (len(devs) == 1 and args.node_shards) else []
        if shards:
            table = [{"G": 1, "ms_per_step": c5w["ms_per_step"], "route_ms": c5w["route_ms"],
                      "merge_ms": c5w["merge_ms"], "h2d_GB": c5w["h2d_GB"], "d2h_GB": c5w["d2h_GB"],
                      "gpu_busy_ms": c5w["gpu_busy_ms"]}]
            for G in shards:
                # each G in a child process given 4 x G hardware queues -- what a G-GPU node gives this pipeline
                # (the HIP runtime's 4 per device): the exchange's per-shard compute, H2D, D2H and peer-copy streams
                # then keep queues of their own, as they do with one shard per GPU (at 4 queues for G shards on one
                # device the copies of different shards serialise behind each other's kernels: profiles/r06/
                # ab_node_queues.sh, G = 2: 905 ms at 4 queues, 728 at 8, 609 at 16)
                r = node_child(args, G, thr)
                if "error" in r:
                    table.append({"G": G, "error": r["error"]})
                    continue
                table.append({"G": G, "ms_per_step": r["ms_per_step"], "route_ms": r["route_ms"],
                              "merge_ms": r["merge_ms"], "h2d_GB": r["h2d_GB"], "d2h_GB": r["d2h_GB"],
                              "gpu_busy_ms": r["gpu_busy_ms"], "shard_rows": r["shard_rows"],
                              "hw_queues": r.get("hw_queues")})
            c5w["node_shards_on_one_gpu"] = {
                "host_threads": thr, "rows": table,
                "note": "G shards (one sg_handle each) mapped onto device 0, each G in a child process with 4 x G HIP "
                        "hardware queues (a G-GPU node's per-device 4): route_ms / merge_ms are the host stages a "
                        "G-GPU node runs, with this box's %d host threads; GPU time and the one PCIe link are "
                        "shared by the G shards" % thr}
    except Exception as e:   # report, never fake
        c5w = {"error": str(e)}
    return c5w


def node_child(args, G, thr):
    """the whole-node pipeline with G shards on device 0, one step, in a child process with min(24, 8 G) hardware
    queues up to G = 4, else 8 (a real node gives each GPU its own queues; on one device, per 1B events
    (profiles/r06/ab_node_queues.sh): G = 2 609 ms at 16 queues (905 at 4), G = 4 644 ms at 24 / 748 at 16 / 890 at 8,
    G = 8 1036 ms at 8 / 1358 at 16 / 2508 at 24 / 2642 at 32 -- its 32 streams oversubscribe the device's queues);
    SG_NODE_CHILD_QUEUES overrides it"""
    cmd = [sys.executable, os.path.abspath(__file__), "--node-only", "--c5-node-steps", "1",
           "--c5-node-devices", ",".join(["0"] * G), "--node-threads", str(thr), "--node-shards", ""]
    if args.c5_events:
        cmd += ["--c5-events", str(args.c5_events)]
    env = {k: v for k, v in os.environ.items() if k not in TORCHRUN_ENV and not k.startswith("TORCHELASTIC")}
    env["GPU_MAX_HW_QUEUES"] = os.environ.get("SG_NODE_CHILD_QUEUES", str(min(24, 8 * G) if G <= 4 else 8))
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "shards child timed out (900 s)"}
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"shards child exit {p.returncode}: {p.stderr[-800:]}"}
    r = json.loads(lines[-1])["whole_node"]
    if isinstance(r, dict):
        r["hw_queues"] = int(env["GPU_MAX_HW_QUEUES"])
    return r


def whole_node_child(args, ws):
    """the whole-node measurement in a child process (a fresh interpreter, not an exec of this one): rank 0 of an
    N-GPU job drives every GPU of the node from it, and a fault on that path costs only this entry"""
    devs = args.c5_node_devices or ",".join(str(g) for g in range(ws))
    thr = args.node_threads or max(16, min(16 * ws, len(os.sched_getaffinity(0))))
    cmd = [sys.executable, os.path.abspath(__file__), "--node-only", "--c5-node-steps", str(args.c5_node_steps),
           "--c5-node-devices", devs, "--node-threads", str(thr), "--node-shards", args.node_shards if ws == 1 else ""]
    if args.c5_events:
        cmd += ["--c5-events", str(args.c5_events)]
    env = {k: v for k, v in os.environ.items() if k not in TORCHRUN_ENV and not k.startswith("TORCHELASTIC")}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "whole-node child timed out (900 s)"}
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"whole-node child exit {p.returncode}: {p.stderr[-800:]}"}
    c5w = json.loads(lines[-1])["whole_node"]
    if isinstance(c5w, dict):
        c5w["process"] = "child"
    return c5w



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed steps of the headline (one step = the whole C5 stream)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C5", help="headline: C5 (BASELINE configs[4], the metric's config) or a "
                                                   "single-push config (C2, C3b, ...)")
    ap.add_argument("--events", type=int, default=0, help="single-push headline: events per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="events for the CPU baseline (default per config: ~5-20 s of oracle work)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=16, help="processes for the key-sharded CPU baseline")
    ap.add_argument("--c5-events", type=int, default=0, help="events of the C5 stream (default 1e9)")
    ap.add_argument("--c5-push-rows", type=int, default=500_000_000)
    ap.add_argument("--c5-node-steps", type=int, default=2,
                    help="steps of the 1B-event C5 stream through the node pipeline, rank 0 driving every GPU (0: skip)")
    ap.add_argument("--c5-node-devices", default="", help="devices of the whole-node pipeline (default: one per rank)")
    ap.add_argument("--node-shards", default="2,4,8",
                    help="N = 1 only: the whole-node pipeline with G shards mapped onto device 0, one step each -- the "
                         "host stages (route, merge) of a G-GPU node measured on one GPU ('' to skip)")
    ap.add_argument("--node-threads", type=int, default=0, help="host threads of the node pipeline (0: 16 per GPU)")
    ap.add_argument("--other-configs", default="C2,C1,C3b,C3c,C4,PP",
                    help="BASELINE configs measured beside the headline (one GPU, rank 0; '' to skip)")
    ap.add_argument("--other-steps", type=int, default=3)
    ap.add_argument("--stream-configs", default="C3c,C3c+bounded",
                    help="sub-lines pushed as 2-push streams with state carried (+bounded: bounded lateness 0 ms)")
    ap.add_argument("--pmc", default="", help="rocprofv3 PMC summary of this command (default profiles/r05/<cfg>_pmc.json)")
    ap.add_argument("--node-child", type=int, default=-1,
                    help="run the whole-node pipeline in a child process (-1: when N > 1, so a fault on the multi-GPU "
                         "exchange path cannot take the headline line with it)")
    ap.add_argument("--node-only", action="store_true", help=argparse.SUPPRESS)   # (the child's mode)
    args = ap.parse_args()
    if args.node_only:
        print(json.dumps({"whole_node": whole_node_block(args, 1, 0, torch.device("cuda", 0))}))
        return

    ws, rank, local = dist_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:   # timing reductions only (no data-path collective): gloo, host tensors
        import torch.distributed as dist
        dist.init_process_group("gloo")
    cfg = args.config
    if not args.cpu_sample:
        args.cpu_sample = CPU_SAMPLE.get(cfg, 12_000_000)
    num, n_cfg, keys, rate = synth.CONFIGS[synth._base(cfg)]

    if cfg == "C5":
        # ---- value: the metric's config, inputs resident in HBM: ONE 1B-event, 1M-key stream sharded by key hash
        # over the ranks (strong scaling), pushed in 500M-row batches with carried state
        head = c5_stream(rank, ws, dev, args.steps, args.warmup, args.c5_events, args.c5_push_rows)
        value, ms_step = head["value"], head["ms_per_step"]
        roof = head.pop("roofline")
        n, matches = head["events"], head["matches"]
        scaling = "strong"
        conf = {"workload": head["workload"], "events_per_step": head["events"], "keys": keys, "rate_events_per_ms": rate,
                "matches_per_step": head["matches"], "push_rows": head["push_rows"],
                "parallelism": f"key-sharded x{ws} (mix64(key) mod N, no collective)"}
        pmc_cfg = "C5"
    else:
        n = args.events or min(n_cfg, 100_000_000)
        m = measure_push(cfg, rank, n, keys, rate, dev, args.steps, args.warmup, sync_ranks=ws > 1)
        ms_step = m["elapsed"] * 1000.0 / args.steps
        value = ws * n * args.steps / m["elapsed"]
        matches = m["matches"]
        roof = roofline_of(cfg, n, matches, m["kern"], m["stage"])
        scaling = "weak"
        conf = {"workload": f"{cfg}: " + synth.QUERIES[cfg], "events_per_gpu_per_step": n, "keys_per_gpu": keys,
                "rate_events_per_ms": rate, "matches_per_gpu_per_step": int(matches),
                "spilled_units": int(m["spilled"]), "parallelism": f"key-sharded x{ws} (no collective)"}
        pmc_cfg = cfg
    # ---- whole node: the same 1B-event C5 stream from pinned host memory through the node pipeline,
    # rank 0 driving every GPU of the job; PCIe-bound, reported beside `value` (never `value`)
    c5w = None
    if args.c5_node_steps > 0:
        if rank == 0:
            child = args.node_child if args.node_child >= 0 else int(ws > 1)
            c5w = whole_node_child(args, ws) if child else whole_node_block(args, ws, local, dev)
        barrier()
    if rank != 0:
        return
    attach_traffic(roof, args.pmc or os.path.join(PMC_DIR, pmc_cfg + "_pmc.json"), pmc_cfg,
                   n if pmc_cfg != "C5" else roof_events(roof))
    cpu = None
    if not args.no_cpu:
        hi = host_info()
        try:
            ccfg = cfg
            r, nm, dt = cpu_baseline(ccfg, args.cpu_sample, keys, rate)
            cpu = {"value": round(r, 1), "unit": "events/s", "cores": 1, "kind": "port",
                   "nproc": hi["nproc"], "cpu_model": hi["cpu_model"],
                   "sample": f"first {args.cpu_sample} events of {ccfg} ({keys} keys, {rate}/ms), oracle C++ "
                             f"restatement of the reference state processors, single thread, {nm} matches, {dt:.1f}s"}
            wk = max(1, min(args.cpu_workers, os.cpu_count() or 1))
            partitioned = ccfg[:2] in ("C2", "C3", "C5")   # C1 / C4 are single runtimes
            if partitioned and wk > 1:
                r2, nm2, dt2 = cpu_baseline_multicore(ccfg, args.cpu_sample, keys, rate, wk)
                cpu["multi_core"] = {"value": round(r2, 1), "cores": wk,
                                     "sample": f"same rows key-sharded over {wk} processes, {nm2} matches, {dt2:.1f}s"}
        except Exception as e:  # report, never fake
            cpu = {"value": None, "unit": "events/s", "cores": 1, "kind": "port", "sample": f"failed: {e}",
                   "nproc": hi["nproc"], "cpu_model": hi["cpu_model"]}
    others = {}
    if args.other_configs:
        for oc in [c for c in args.other_configs.split(",") if c and c != cfg]:
            try:
                others[oc] = config_line(oc, dev, args.other_steps, 1, not args.no_cpu)
            except Exception as e:   # report, never fake
                others[oc] = {"error": str(e)}
    if args.stream_configs:
        for sc in [c for c in args.stream_configs.split(",") if c]:
            lat = -1
            name = sc
            if sc.endswith("+bounded"):
                sc, lat = sc[:-len("+bounded")], 0
            try:
                others[name + "_stream"] = stream_line(sc, dev, args.other_steps, 1, lateness=lat)
            except Exception as e:   # report, never fake
                others[name + "_stream"] = {"error": str(e)}
    line = {
        "metric": "events/sec (whole node) for partitioned pattern query at 1/2/4/8 GPUs; % HBM peak",
        "value": round(value, 1), "unit": "events/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (SplitMix64 generator, SURVEY.md §8d), inputs resident in HBM; matches "
                               "projected in HBM (zero-copy sg_device_records)",
        "config": conf,
        "cpu_baseline": cpu,
        "configs": others,
        "source_hash": source_hash(pmc_cfg),
        "whole_node": c5w,   # (last: the driver stores the line's tail)
        "roofline": roof,
    }
    print(json.dumps(line))


def roof_events(roof):
    """events of one push the roofline was taken on (C5: rank 0's share of the stream over its pushes)"""
    return int(roof.get("push_events", 0))


if __name__ == "__main__":
    main()
