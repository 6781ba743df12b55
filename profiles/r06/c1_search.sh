#!/bin/bash
# C1's forward search with its loads issued eight rows at a time: every test of the unpartitioned search, then the C1
# sub-line
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-c1s}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_time_regression.py tests/test_walker_paths.py tests/test_full_size.py tests/test_gpu_parity.py \
  -k "unpartitioned or c1 or C1 or long_completion or walker or kat" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs C1,C2 --stream-configs= \
  --other-steps 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('C5', d['ms_per_step'])
for k,v in d['configs'].items(): print(k, v.get('ms_per_push'), v.get('matches'), v.get('kernels_ms'))
"
