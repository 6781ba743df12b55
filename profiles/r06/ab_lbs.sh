#!/bin/bash
# C5 headline with 256 / 128 / 64 / 32 supergroups in the wide partition's pass 1 (measured with a since-removed
# SG_DEBUG_P1_LBS hook = 0..3; the default is now 64 supergroups)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-ablbs}
mkdir -p $OUT
for e in ${LBS:-0 1 2 3 0}; do
  SG_DEBUG_P1_LBS=$e timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs= \
    --stream-configs= > $OUT/lbs$e.json 2> $OUT/lbs$e.err || { echo "bench failed"; tail -20 $OUT/lbs$e.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/lbs$e.json').read().strip().splitlines()[-1])
r=d['roofline']; k=r.get('kernels_ms')
print('lbs+$e', d['ms_per_step'], {x: k[x] for x in ('part_hist','part_group','part_split','group_walk','gw_project')})"
done
