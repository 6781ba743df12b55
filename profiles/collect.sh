#!/bin/bash
# Collect the committed evidence for one round (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the bench command (per-kernel durations)
#   2. separate --pmc passes (MI355X_MICROARCH.md: no multiplexing; <=4 TCC counters per pass):
#      FETCH_SIZE | WRITE_SIZE | TCC_EA0_RDREQ by request size
# usage: profiles/collect.sh <outdir> [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 -u bench.py --steps 3 --warmup 1 --no-cpu "$@" > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$out/pmc$i" -o run -- \
    python3 -u bench.py --steps 1 --warmup 1 --no-cpu "$@" > "$out/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo done
