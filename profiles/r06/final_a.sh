#!/bin/bash
# Final tree, call 1: every test of the wide-partition / group-walker path (the last kernel change was the wide
# partition's supergroup count), then the C5 trace + PMC collection.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/fin2
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_wide_partition.py tests/test_group_walk.py tests/test_c5_headline.py tests/test_push_size.py \
  tests/test_time_regression.py::test_closed_form_wide_partition_jitter tests/test_full_size.py -k "not C3 and not PP and not c1" \
  > $OUT/wide_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/wide_tests.log; exit 1; }
tail -2 $OUT/wide_tests.log
bash profiles/r06/collect.sh gpurun_out/pmcG C5
