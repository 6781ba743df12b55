#!/bin/bash
# PMC passes over one bench step (each counter group in its own run, per MI355X_MICROARCH.md).
# usage: profiles/pmc_walk.sh <outdir> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
mkdir -p "$out"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/pass$i" -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
