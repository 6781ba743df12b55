#!/bin/bash
# rocprofv3 kernel trace + stats of one bench config (one push per step): per-kernel durations
# usage: profiles/r04/ktrace.sh <outdir> <cfg> [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; cfg=$2; shift 2
d="$out/$cfg"; mkdir -p "$d"
args="--config $cfg --steps 2 --warmup 1 --no-cpu --other-configs= --c5-node-steps 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -o run -- \
  python3 -u bench.py $args > "$d/trace.log" 2>&1 || { echo "$cfg trace failed"; tail -5 "$d/trace.log"; exit 1; }
f=$(find "$d/trace" -name "run_kernel_stats.csv" | head -1)
cp "$f" "$d/kernel_stats.csv" && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$d/kernel_stats.csv')))
for r in rows[:14]: print('%-60s %6s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
