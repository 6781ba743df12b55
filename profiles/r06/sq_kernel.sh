#!/bin/bash
# SQ counters of one kernel (regex) over one C5 headline step, one rocprofv3 --pmc pass per counter group
# (<= 8 SQ counters per pass), then FETCH_SIZE / WRITE_SIZE.  usage: sq_kernel.sh <outdir> <kernel-regex> [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; shift; rx=$1; shift
mkdir -p "$out"
args="--steps 1 --warmup 0 --no-cpu --c5-node-steps 0 --other-configs= $*"
i=0
for g in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $g --kernel-include-regex "$rx" --output-format csv -d "$out/pass$i" -o run -- \
    python3 -u bench.py $args > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/pass*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(f"{k:24s} {tot[k]:.4g}  (rows {n[k]})")
PY
