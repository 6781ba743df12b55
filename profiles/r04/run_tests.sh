#!/bin/bash
# run a subset of the GPU tests: profiles/r04/run_tests.sh <outdir> <pytest args...>
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -p no:cacheprovider "$@" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
