#!/usr/bin/env python3
"""Benchmark: whole-node events/sec of the partitioned pattern query on MI355X.

Workload (BASELINE.json configs[1]):
  partition with (symbol of StockStream) begin
    from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
    select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;
  100M synthetic events per GPU (SplitMix64 generator, siddhi_amd/synth.py), 10k keys, 1000 events/ms.
A step = one sg_push of the whole 100M-event batch (inputs already resident in HBM) through the HIP
pipeline (predicate-eval bitmasks -> key partition -> per-key walker count -> scan -> walker write) on a
fresh state.
Multi-GPU (one process per GPU, torchrun): weak scaling, rank r owns the disjoint key range
[r*K, (r+1)*K) with its own 100M-event stream; no data-path collective (keys never interact).

Prints ONE JSON line (rank 0).  Roofline figures use algorithmic bytes.
"""
import argparse
import json
import os
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


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


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
    """The same oracle on all host cores the box grants this job: rows sharded by partition key across
    worker processes (keys never interact), each shard keeping its global event indices."""
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


def path_traffic(profile_json, n, cfg):
    """HBM-side bytes of one push from the committed PMC summary (profiles/collect.sh + summarize.py):
    every kernel of the path (torch's synthetic-data kernels excluded), per dispatch."""
    try:
        with open(profile_json) as f:
            prof = json.load(f)
    except OSError:
        return None, None
    if prof.get("workload") != cfg or prof.get("events") != n:
        return None, None
    tot = 0.0
    for k, d in prof["kernels"].items():
        if k.startswith("torch::") or k.startswith("__amd_rocclr"):
            continue
        tot += d.get("read_bytes_per_dispatch", 0.0) * d.get("dispatches_per_push", 1)
        tot += d.get("write_bytes_per_dispatch", 0.0) * d.get("dispatches_per_push", 1)
    return tot, profile_json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--events", type=int, default=0, help="events per GPU per step (default: config size, max 1e8)")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="events for the CPU baseline (default per config: ~5-20 s of oracle work; C4 60k -- the "
                         "oracle walks ~5k partials per event)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=16, help="processes for the key-sharded CPU baseline")
    ap.add_argument("--host-input", action="store_true",
                    help="columns in pinned host memory, pushed through the chunked ingress (PCIe-inclusive rate; "
                         "never the headline value)")
    ap.add_argument("--ingress-rows", type=int, default=0, help="ingress chunk rows for --host-input (0 = engine default, -1 = one copy)")
    ap.add_argument("--profile", default=os.path.join(ROOT, "profiles", "r01", "c2_profile.json"),
                    help="committed PMC summary the roofline traffic is read from")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    cfg = args.config
    if not args.cpu_sample:   # ~5-20 s of single-thread oracle work per config (measured rates)
        args.cpu_sample = {"C1": 1_000_000, "C3b": 6_000_000, "C3c": 3_000_000, "C4": 60_000,
                           "C5": 3_000_000}.get(cfg, 12_000_000)
    num, n_cfg, keys, rate = synth.CONFIGS[cfg[:2]]
    n = args.events or min(n_cfg, 100_000_000)

    # ---- synthetic rows of this rank's key shard, generated in HBM
    # (each rank's keys are its own dense ids 0..K-1: the router re-densifies per rank, siddhi_amd/router.py)
    g = synth.generate_torch(cfg, rank * n, n, dev, keys=keys, rate=rate)
    key = g["key"].to(torch.int32) if "key" in g else torch.zeros(n, dtype=torch.int32, device=dev)
    if cfg.startswith("C4"):     # S(id, seq) rows only (the Tick stream's column is never read)
        cols = [g["id"], g["seq"], torch.zeros(n, dtype=torch.int32, device=dev)]
    elif cfg.startswith("C3"):
        cols = [g["id"], key, g["v"], g["w"]]
    else:
        cols = [g["id"], key, g["price"]]
    torch.cuda.synchronize()

    keep = []
    if args.host_input:
        # pinned host columns; chunks are consecutive sub-pushes, so the handle carries state (reset per step)
        h, nfa = make_handle(cfg, no_carry=0, ingress_rows=args.ingress_rows)

        def pinned(t):
            a = t.cpu().numpy()
            p = N.PinnedArray(len(a), a.dtype)
            p.array[:] = a
            keep.append(p)
            return p.array.ctypes.data
        batch = N.make_batch(n, rank * n, pinned(g["ts"]), 0, pinned(key), [pinned(c) for c in cols],
                             [0] * len(cols), 0, keys, keep)
    else:
        h, nfa = make_handle(cfg)   # each step is a complete stream: no state carried between steps
        batch = N.make_batch(n, rank * n, g["ts"].data_ptr(), 0, key.data_ptr(), [c.data_ptr() for c in cols],
                             [0] * len(cols), 1, keys, keep)
    stream = torch.cuda.current_stream()
    h.check(h.lib.sg_set_stream(h.h, stream.cuda_stream))

    def step():
        h.reset()
        h.push(batch)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    stage = np.zeros(5)
    matches = 0
    spilled = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        t = h.timing()
        stage += [t.pred_ms, t.partition_ms, t.match_ms, t.output_ms, t.total_ms]
        matches = h.pending() if args.host_input else t.matches   # (timing covers the last ingress chunk)
        spilled = t.spilled_units
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        dist.barrier()
    stage /= args.steps
    if rank != 0:
        return
    ms_step = elapsed * 1000.0 / args.steps
    value = ws * n * args.steps / elapsed

    # algorithmic bytes: predicate pass 4.125 B/event (price read + condition bit);
    # whole path 16.125 B/event (ts 8 + key 4 + price 4 + bit) + 36 B/match (C1: no key, 12.125);
    # C4 (no local predicate): ts 8 + id 8 B/event + 28 B/emission
    pred_bytes = 4.125 * n
    per_ev, per_m = {"C1": (12.125, 36.0), "C4": (16.0, 28.0)}.get(cfg[:2], (16.125, 36.0))
    path_bytes = per_ev * n + per_m * matches
    stages = {"pred_eval_ms": stage[0], "key_partition_ms": stage[1], "walk_count_scan_ms": stage[2],
              "walk_write_ms": stage[3], "kernels_total_ms": stage[4]}
    names = ["pred_eval_ms", "key_partition_ms", "walk_count_scan_ms", "walk_write_ms"]
    dom = names[int(np.argmax(stage[:4]))]
    path_gbs = path_bytes / (stage[4] * 1e-3) / 1e9
    pred_gbs = pred_bytes / (stage[0] * 1e-3) / 1e9 if stage[0] > 0 else 0.0
    roof = {"bound": "hbm", "achieved": round(path_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(path_gbs / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "whole NFA path (all kernels of one push; dominant stage: %s)" % dom,
            "pred_eval_pass": {"achieved": round(pred_gbs, 1), "frac": round(pred_gbs / HBM_PEAK_GBS, 4),
                               "bytes_per_event": 4.125},
            "stages_ms": {k: round(v, 4) for k, v in stages.items()}}
    if args.host_input:
        roof["note"] = "stages_ms / achieved cover the last ingress chunk's kernels only"
    if cfg.startswith("C4"):
        roof["pred_eval_pass"] = None   # no local predicate: the path starts at the role/value pass
    traffic, tsrc = path_traffic(args.profile, n, cfg)
    if traffic is not None:
        roof["traffic"] = round(traffic / 1e9, 3)
        roof["traffic_unit"] = "GB per push (L2-side EA requests incl. Infinity-Cache hits; %s)" % os.path.relpath(tsrc, ROOT)
    cpu = None
    if not args.no_cpu:
        try:
            r, nm, dt = cpu_baseline(cfg, args.cpu_sample, keys, rate)
            cpu = {"value": round(r, 1), "unit": "events/s", "cores": 1, "kind": "port",
                   "sample": f"first {args.cpu_sample} events of {cfg} ({keys} keys, {rate}/ms), oracle C++ "
                             f"restatement of the reference state processors, single thread, {nm} matches, {dt:.1f}s"}
            wk = max(1, min(args.cpu_workers, os.cpu_count() or 1))
            partitioned = cfg[:2] in ("C2", "C3", "C5")   # C1 / C4 are single runtimes
            if partitioned and wk > 1:
                r2, nm2, dt2 = cpu_baseline_multicore(cfg, args.cpu_sample, keys, rate, wk)
                cpu["multi_core"] = {"value": round(r2, 1), "cores": wk,
                                     "sample": f"same rows key-sharded over {wk} processes, {nm2} matches, {dt2:.1f}s"}
        except Exception as e:  # report, never fake
            cpu = {"value": None, "unit": "events/s", "cores": 1, "kind": "port", "sample": f"failed: {e}"}
    line = {
        "metric": "events/sec (whole node) for partitioned pattern query at 1/2/4/8 GPUs; % HBM peak",
        "value": round(value, 1), "unit": "events/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (SplitMix64 generator, SURVEY.md §8d), " +
        ("in pinned host memory: PCIe-inclusive chunked ingress (not the headline figure)" if args.host_input
         else "resident in HBM"),
        "config": {"workload": f"{cfg}: " + synth.QUERIES[cfg], "events_per_gpu_per_step": n,
                   "keys_per_gpu": keys, "rate_events_per_ms": rate, "matches_per_gpu_per_step": int(matches),
                   "spilled_units": int(spilled),
                   "parallelism": f"key-sharded x{ws} (no collective)"},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))


if __name__ == "__main__":
    main()
