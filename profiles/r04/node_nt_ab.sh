#!/bin/bash
# A/B of the node's streaming-store switches on ONE box (host-stage times move between boxes):
# profiles/r04/node_nt_ab.sh <outdir>
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; mkdir -p "$out"
for m in 1 3 7 3 1; do
  SG_NODE_NT=$m timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --other-configs= --no-cpu --c5-node-steps 1 \
    > "$out/nt$m.json" 2> "$out/nt$m.err" || { echo "nt$m failed"; tail -3 "$out/nt$m.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/nt$m.json')); wn=d['whole_node']
print('SG_NODE_NT=$m', [(r['G'], r['ms_per_step'], r['route_ms'], r['merge_ms']) for r in wn['node_shards_on_one_gpu']['rows']])"
done
