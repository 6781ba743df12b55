#!/bin/bash
# Node pipeline (1B C5 stream from pinned host memory): G = 1 and the G = 2 exchange on one device, at the HIP
# runtime's default hardware queues per process and with more of them
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abq
for q in ${QS:-4 8 16}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 500 python -u bench.py --steps 1 --warmup 0 --no-cpu --other-configs= --stream-configs= \
    --c5-node-steps 2 --node-shards 2 > gpurun_out/abq/q$q.json 2> gpurun_out/abq/q$q.err || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/abq/q$q.json').read().strip().splitlines()[-1])
w=d['whole_node']; print('queues=$q G=1', w['ms_per_step'], 'h2d', w['h2d_GB'], 'd2h', w['d2h_GB'])
for s in w.get('node_shards_on_one_gpu', {}).get('rows', []): print('   G=%s' % s['G'], s['ms_per_step'], 'h2d', s['h2d_GB'], 'd2h', s['d2h_GB'], 'busy', s['gpu_busy_ms'])"
done
