#!/usr/bin/env python3
"""Summarise profiles/r06/collect.sh output (C5 = the 1B stream, per push): per engine mark (the kernel groups the engine times with HIP events,
sg_timing.kernel_ms) the average duration per push from the kernel trace and the HBM-side bytes per push from the
FETCH_SIZE / WRITE_SIZE passes.  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half the bytes of 128-B
streaming reads (doubled here) and WRITE_SIZE is exact for 16-B/lane streaming stores; both are L2-side
counters, so Infinity-Cache hits are included (an upper bound on DRAM bytes).

usage: profiles/r06/summarize.py <collect dir> <config>   (pushes per run are read off the run's bench line)"""
import csv
import glob
import hashlib
import json
import os
import re
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

MARKS = [   # kernel name pattern -> engine mark (siddhi_amd/csrc: h->kbeg names)
    (r"k_gwalk", "group_walk"), (r"k_gw_redo", "gw_redo"), (r"k_gw_count", "gw_count"), (r"k_gtile_count", "gw_tiles"),
    (r"k_gscan_project", "gw_project"),
    (r"k_part1b", "part_split"), (r"k_hist_wide", "part_hist"), (r"k_carry_", "carry"), (r"k_pp_wsum", "wait_sum"),
    (r"k_once_first|k_once_bind|k_once_second|k_once_finish", "once_match"), (r"k_once_project", "once_order"),
    (r"k_fgw_proj", "fgw_project"), (r"k_fgw_plan|k_fgw_cb", "fgw_plan"), (r"k_fgw\b|k_fgw<", "fgw_walk"),
    (r"k_sq_spec", "sequence_lanes"), (r"k_sq_fix", "sequence_fix"), (r"k_pp_lanes", "partial_lanes"),
    (r"k_pred_simple|k_pred\b", "pred"), (r"k_pack\b", "pack"), (r"onesweep", "key_sort"),
    (r"k_part1_hist", "part_hist"), (r"k_part2_hist", "part_hist2"), (r"k_part1<", "part_group"),
    (r"k_part2<|k_part_segs", "part_key"),
    (r"k_bounds\b", "bounds"), (r"k_units\b|k_rowmap\b", "units"), (r"k_transpose\b", "tile_transpose"),
    (r"k_walk_t<[^>]*false>", "walk_count"), (r"k_walk_t<[^>]*true>", "walk_record"),
    (r"k_walk<[^>]*false, true>", "walk_count"), (r"k_walk<[^>]*true, true>", "walk_record"),
    (r"k_project\b", "project"), (r"k_carry_copy\b|k_nge_carry", "carry"), (r"k_nge_blocks|k_nge\b", "nge_search"),
    (r"k_route\b", "route"), (r"k_segments\b", "key_sort"), (r"k_nfa_units|k_unit_", "nfa_units"),
    (r"k_nfa\b", "nfa_keys"), (r"k_sortkeys|k_gather\b|k_em_", "match_order"), (r"k_abs_rows|k_abs_init", "abs_roles"),
    (r"k_abs_keys|k_abs_rkill|k_abs_kill", "abs_sort_kill"), (r"k_abs_decide", "abs_decide_scan"),
    (r"k_abs_slot|k_abs_heads|k_abs_write|k_abs_last", "abs_write"),
    (r"scan|lookback", "scans"), (r"radix_sort|histogram", "key_sort"),
]


def mark_of(name):
    if "at::native" in name or "at::" in name[:40]:
        return None   # torch's synthetic-data kernels (outside the timed path)
    if "__amd_rocclr" in name:
        return "runtime_fill_copy"
    for rx, m in MARKS:
        if re.search(rx, name):
            return m
    return name.split("(")[0][:60]


def main(d, cfg):
    log = open(os.path.join(d, "trace.log")).read().strip().splitlines()
    line = json.loads([l for l in log if l.startswith("{")][-1])
    runs = line["steps"] + line["warmup"]
    if cfg == "C5":   # the stream: every step pushes rank 0's share in push_rows batches
        per_step = -(-line["config"]["events_per_step"] // line["config"]["push_rows"])
        pushes, events = runs * per_step, line["roofline"]["push_events"]
    else:
        pushes, events = runs, line["config"]["events_per_gpu_per_step"]
    out = {"workload": cfg, "kernels": {}, "pushes_per_run": pushes}
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(d, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            m = mark_of(r["Kernel_Name"])
            if m:
                dur[m] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    byt = defaultdict(float)
    for i, scale in ((1, 2.0), (2, 1.0)):   # FETCH_SIZE x2 (half-counted 128-B reads), WRITE_SIZE exact
        for f in glob.glob(os.path.join(d, "pmc%d" % i, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                m = mark_of(r["Kernel_Name"])
                if m:
                    byt[m] += float(r["Counter_Value"]) * 1024.0 * scale
    for m in sorted(set(dur) | set(byt), key=lambda k: -dur.get(k, 0)):
        out["kernels"][m] = {"avg_us_per_push": round(dur.get(m, 0) / pushes, 2),
                             "bytes_per_push": byt.get(m, 0.0) / pushes}
    sys.path.insert(0, ROOT)
    import bench   # noqa: E402  (source hash of the measured tree)
    out["source_hash"] = bench.source_hash(cfg)
    try:
        out["git_head"] = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                         text=True).stdout.strip() or None
    except Exception:
        out["git_head"] = None
    out["events"] = events
    out["bench_line_of_trace_run"] = {k: line[k] for k in ("value", "ms_per_step")}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
