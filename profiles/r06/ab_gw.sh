#!/bin/bash
# A/B of the group walker's LDS geometry (rows per thread per chunk x ring entries) on the C5 headline
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab2
for cfg in ${CFGS:-8:8 12:8 10:8}; do
  set -- ${cfg/:/ }
  SG_DEBUG_GW_PT=$1 SG_DEBUG_GW_CAP=$2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs= > gpurun_out/ab2/pt$1_cap$2.json 2>gpurun_out/ab2/pt$1_cap$2.err || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/ab2/pt$1_cap$2.json').read().strip().splitlines()[-1])
r=d['roofline']; print('PT=$1 cap=$2', d['ms_per_step'], {k:v for k,v in list(r['kernels_ms'].items())[:5]})"
done
