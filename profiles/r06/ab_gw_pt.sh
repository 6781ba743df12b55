#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab1
for pt in 16 8 4; do
  SG_DEBUG_GW_PT=$pt timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs= > gpurun_out/ab1/pt$pt.json 2>gpurun_out/ab1/pt$pt.err || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/ab1/pt$pt.json').read().strip().splitlines()[-1])
r=d['roofline']; print('PT=$pt', d['ms_per_step'], {k:v for k,v in list(r['kernels_ms'].items())[:4]})"
done
