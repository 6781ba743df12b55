#!/bin/bash
# sequence-lane kernel time per SG_SQ_ROWS (rows per speculative unit) on one box: profiles/r04/seq_ab.sh <outdir>
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; mkdir -p "$out"
for r in 382 192 600 1000 1600 382; do
  SG_SQ_ROWS=$r timeout -k 10 300 python -u bench.py --config C3b --steps 3 --warmup 1 --no-cpu --other-configs= \
    --c5-node-steps 0 > "$out/r$r.json" 2> "$out/r$r.err" || { echo "r$r failed"; tail -3 "$out/r$r.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/r$r.json')); k=d['roofline']['kernels_ms']
print('SG_SQ_ROWS=$r', 'push ms', d['ms_per_step'], 'sequence_lanes', k.get('sequence_lanes'), 'fix', k.get('sequence_fix'))"
done
