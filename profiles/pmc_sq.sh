#!/bin/bash
# SQ-side evidence for the walker / general-machine kernels (occupancy, stall split, instruction mix) plus
# FETCH/WRITE passes, one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: <=8 SQ, <=4 TCC per
# pass; no multiplexing).  usage: profiles/pmc_sq.sh <outdir> <kernel-regex> -- [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift; rx=$1; shift
[ "$1" == "--" ] && shift
mkdir -p "$out"
timeout -s KILL 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
i=0
for g in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "$rx" --output-format csv -d "$out/pass$i" -o run -- \
    python3 -u bench.py --steps 1 --warmup 1 --no-cpu --c5-stream-steps 0 "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 -u bench.py --steps 2 --warmup 1 --no-cpu --c5-stream-steps 0 "$@" > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
echo done
