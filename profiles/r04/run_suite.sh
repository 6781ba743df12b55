#!/bin/bash
# r04: handle-leak test first (fresh child process), then the whole GPU suite with no early torch initialisation
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 700 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_handle_leaks.py > $OUT/leaks.log 2>&1 || { echo "leak test failed"; tail -40 $OUT/leaks.log; exit 1; }
tail -2 $OUT/leaks.log
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  -s --deselect tests/test_handle_leaks.py tests/ > $OUT/tests.log 2>&1 || { echo "suite failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
