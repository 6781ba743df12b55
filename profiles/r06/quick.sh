#!/bin/bash
# r06 quick GPU check: C5-path parity tests (wide partition, C5 time regression, snapshot, headline 60M), then a short
# C5 headline bench with per-kernel HIP-event times.  Usage: quick.sh <out-name>
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_wide_partition.py tests/test_c5_headline.py "tests/test_time_regression.py" -k "wide or C5 or c5 or headline" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --c5-node-steps 0 --other-configs C2 --other-steps 2 \
  > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "
import json,sys
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'])
r=d['roofline']; print('dominant', r['kernel'], r['kernel_ms'], 'frac', r['frac']); print(r.get('kernels_ms'))
"
