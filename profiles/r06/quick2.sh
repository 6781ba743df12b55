#!/bin/bash
# r06: group-walk / headline / bounded-lateness tests, then the C5 headline and the streaming C3c sub-lines
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-quick2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_group_walk.py tests/test_c5_headline.py tests/test_partial_lanes.py -k "group or headline or bounded" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs= \
  --stream-configs ${STREAMS:-C3c,C3c+bounded} --other-steps 2 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'])
r=d['roofline']; print('dominant', r['kernel'], r['kernel_ms'], 'frac', r['frac']); print(r.get('kernels_ms'))
for k,v in d['configs'].items(): print(k, v.get('ms_per_stream', v.get('ms_per_push')), v.get('matches'), v.get('kernels_ms_per_stream', v.get('error')))
"
