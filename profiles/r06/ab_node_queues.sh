#!/bin/bash
# Node pipeline (1B C5 stream from pinned host memory) with G shards on one device, per hardware-queue count of the
# shards' child process (SG_NODE_CHILD_QUEUES; bench.py's default is min(16, 4 G))
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abq
for q in ${QS:-8 16 24}; do
  SG_NODE_CHILD_QUEUES=$q timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu --other-configs= --stream-configs= \
    --c5-node-steps 1 --node-shards ${SHARDS:-4,8} > gpurun_out/abq/q$q.json 2> gpurun_out/abq/q$q.err || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/abq/q$q.json').read().strip().splitlines()[-1])
w=d['whole_node']
for s in w.get('node_shards_on_one_gpu', {}).get('rows', []): print('queues=$q G=%s' % s['G'], s['ms_per_step'], 'h2d', s['h2d_GB'], 'd2h', s['d2h_GB'], s.get('hw_queues'))"
done
