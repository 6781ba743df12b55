#!/bin/bash
# kernel trace of a short bench run -> per-kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --c5-stream-steps 0 "$@" > "$out/bench.log" 2>&1
