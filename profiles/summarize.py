#!/usr/bin/env python3
"""Summarise profiles/collect.sh output into one JSON: per-kernel average duration (kernel trace) and
per-dispatch HBM-side traffic (PMC), plus per-push path totals.

Traffic, per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) = TCC_EA0_RDREQ x 64 B and reports half the bytes of
128-B requests; so read bytes are rebuilt from the request-size classes
(32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B), and write bytes are WRITE_SIZE (exact for 16-B/lane
streaming stores).  Infinity-Cache hits are counted by these L2-side counters, so this is an upper bound on
DRAM bytes."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    n = re.sub(r"^void ", "", n)
    if n.startswith("at::native") or "at::native" in n[:60]:
        return "torch::" + re.sub(r"[^A-Za-z]+", "_", name[40:100])[:40]
    if "rocprim" in n:
        kind = ("onesweep_global_offsets" if "onesweep_global_offsets" in name
                else "onesweep_iteration" if "onesweep_iteration" in name
                else "lookback_init" if "init_lookback" in name else "scan" if "scan_impl" in name else "other")
        return "rocprim::" + kind
    return n


def pmc(d):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return acc, disp


def main(out, workload="C2", events=100_000_000, pushes_traced=4, pushes_pmc=2):
    res = {"workload": workload, "events": events, "kernels": {}}
    trace = defaultdict(list)
    for f in glob.glob(os.path.join(out, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            trace[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    per = defaultdict(dict)
    for k, v in trace.items():
        per[k]["calls_traced"] = len(v)
        per[k]["avg_us"] = round(sum(v) / len(v) / 1000.0, 2)
        per[k]["dispatches_per_push"] = len(v) / pushes_traced
    for i in (1, 2, 3):
        acc, disp = pmc(os.path.join(out, "pmc%d" % i))
        for k, cs in acc.items():
            nd = max(1, len(disp[k]))
            for c, v in cs.items():
                per[k][c.replace("_sum", "") + "_per_dispatch"] = v / nd
    for k, d in per.items():
        if "TCC_EA0_RDREQ_128B_per_dispatch" in d:
            d["read_bytes_per_dispatch"] = (32 * d.get("TCC_EA0_RDREQ_32B_per_dispatch", 0) +
                                            64 * d.get("TCC_EA0_RDREQ_64B_per_dispatch", 0) +
                                            128 * d.get("TCC_EA0_RDREQ_128B_per_dispatch", 0))
        if "WRITE_SIZE_per_dispatch" in d:
            d["write_bytes_per_dispatch"] = d["WRITE_SIZE_per_dispatch"] * 1024.0
        if "FETCH_SIZE_per_dispatch" in d:
            d["fetch_size_bytes_x2_per_dispatch"] = d["FETCH_SIZE_per_dispatch"] * 1024.0 * 2
    res["kernels"] = dict(sorted(per.items(), key=lambda kv: -kv[1].get("avg_us", 0)))
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
