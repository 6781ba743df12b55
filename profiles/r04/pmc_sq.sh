#!/bin/bash
# SQ counters of one bench config (a separate --pmc pass): profiles/r04/pmc_sq.sh <outdir> <cfg>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; cfg=$2; d="$out/$cfg"; mkdir -p "$d"
args="--config $cfg --steps 1 --warmup 1 --no-cpu --other-configs= --c5-node-steps 0"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU \
  --output-format csv -d "$d/sq" -o run -- python3 -u bench.py $args > "$d/sq.log" 2>&1 || { echo "sq pass failed"; tail -5 "$d/sq.log"; exit 1; }
f=$(find "$d/sq" -name "run_counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:50]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0))[:8]:
    print(k, {x: "%.3g" % y for x, y in sorted(c.items())})
PY
