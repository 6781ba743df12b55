#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (or kernel_stats.csv) into per-kernel time stats (CSV on stdout)."""
import csv
import sqlite3
import sys
from collections import defaultdict


def main(path):
    rows = defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute('select name, start, "end" from kernels'):
            rows[name].append(e - s)
    else:
        for r in csv.DictReader(open(path)):
            rows[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in rows.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name[:160], len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 3), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
