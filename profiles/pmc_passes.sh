#!/bin/bash
# Run one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: no multiplexing; <=8 SQ, <=4 TCC).
# usage: profiles/pmc_passes.sh <outdir> <kernel-regex> "<group1>" "<group2>" ... -- [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift; rx=$1; shift
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$out"
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "$rx" --output-format csv -d "$out/pass$i" -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
