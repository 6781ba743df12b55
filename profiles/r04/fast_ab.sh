#!/bin/bash
# FAST lane kernels (chain.h sg_terms_fast) against the general ones on one box: profiles/r04/fast_ab.sh <outdir>
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; mkdir -p "$out"
for cfg in C3c C3b; do
  for v in 0 1 0; do
    SG_LANES_NO_FAST=$v timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu --other-configs= \
      --c5-node-steps 0 > "$out/$cfg.nofast$v.json" 2> "$out/$cfg.nofast$v.err" || { echo "$cfg $v failed"; tail -3 "$out/$cfg.nofast$v.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/$cfg.nofast$v.json')); k=d['roofline']['kernels_ms']
print('$cfg SG_LANES_NO_FAST=$v', 'push ms', d['ms_per_step'], {x: k.get(x) for x in ('partial_lanes', 'sequence_lanes')})"
  done
done
