#!/bin/bash
# A/B of the wide partition's first pass sub-tile (rows per thread) on the C5 headline
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab3
for pt in ${PTS:-4 8 16}; do
  SG_DEBUG_P1_PT=$pt timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs= --stream-configs= > gpurun_out/ab3/p1_$pt.json 2>gpurun_out/ab3/p1_$pt.err || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/ab3/p1_$pt.json').read().strip().splitlines()[-1])
r=d['roofline']; print('P1=$pt', d['ms_per_step'], r['kernels_ms'])"
done
