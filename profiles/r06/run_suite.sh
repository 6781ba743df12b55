#!/bin/bash
# r06: GPU suite in parts (each part one pytest process, its own time limit); part "leak" runs the handle-leak test
# alone in a fresh process first.  Usage: run_suite.sh <out-name> <part>   part = leak | a | b | smoke | <test paths>
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-suite}; shift
mkdir -p $OUT
PART=${1:-a}; shift
PY="python -u -m pytest -x -v --timeout-method thread -m gpu -p no:cacheprovider"
case "$PART" in
  leak)  timeout -k 10 900 $PY --timeout 900 -s tests/test_handle_leaks.py > $OUT/leak.log 2>&1; rc=$? ;;
  a)     timeout -k 10 1000 $PY --timeout 300 --deselect tests/test_handle_leaks.py \
           $(ls tests/test_*.py | awk '$0 < "tests/test_node.py"') > $OUT/a.log 2>&1; rc=$? ;;
  b)     timeout -k 10 1100 $PY --timeout 700 $(ls tests/test_*.py | awk '$0 >= "tests/test_node.py"') "$@" > $OUT/b.log 2>&1; rc=$? ;;
  smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$? ;;
  *)     timeout -k 10 1100 $PY --timeout 700 "$PART" "$@" > $OUT/custom.log 2>&1; rc=$? ;;
esac
tail -5 $OUT/*.log
exit $rc
