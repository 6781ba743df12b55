#!/bin/bash
# partial-lane kernel time per SG_PP_WAVE_CANDS (start rows per wave) on one box: profiles/r04/lanes_ab.sh <outdir>
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; mkdir -p "$out"
for w in 512 128 256 384 512; do
  SG_PP_WAVE_CANDS=$w timeout -k 10 300 python -u bench.py --config C3c --steps 3 --warmup 1 --no-cpu --other-configs= \
    --c5-node-steps 0 > "$out/w$w.json" 2> "$out/w$w.err" || { echo "w$w failed"; tail -3 "$out/w$w.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/w$w.json')); k=d['roofline']['kernels_ms']
print('SG_PP_WAVE_CANDS=$w', 'push ms', d['ms_per_step'], 'partial_lanes', k.get('partial_lanes'))"
done
