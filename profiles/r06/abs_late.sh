#!/bin/bash
# Absence route with late rows: the segmented push (closed form / one-wave sequential pass / closed form) -- parity on
# every absence test, then the k_abs_seq cost at C4's full size with 0, 1, 10, 100 late rows.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-abslate}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_time_regression.py tests/test_absent_closed_form.py tests/test_ingress.py -k "absen or C4 or once" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u profiles/r06/abs_seq_cost.py 0,1,10,100,1000 > $OUT/abs_seq_cost.jsonl 2> $OUT/abs.err || { echo "cost run failed"; tail -20 $OUT/abs.err; exit 1; }
cat $OUT/abs_seq_cost.jsonl
