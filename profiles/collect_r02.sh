#!/bin/bash
# Evidence for one bench line (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the bench command (per-kernel durations, stats CSV)
#   2. separate --pmc passes FETCH_SIZE | WRITE_SIZE (MI355X_MICROARCH.md §HBM: one TCC group per pass)
#   3. profiles/summarize_r02.py -> <out>/summary.json (per engine mark: avg us, HBM bytes per push), stamped with
#      the kernel-source hash bench.py checks before it trusts the traffic figure
# usage: profiles/collect_r02.sh <outdir> <config> [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; cfg=$2; shift 2
mkdir -p "$out"
args="--config $cfg --steps 2 --warmup 1 --no-cpu --whole-node-steps 0 --c5-stream-steps 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 -u bench.py $args > "$out/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$out/trace.log"; exit 1; }
i=0
for g in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $g --output-format csv -d "$out/pmc$i" -o run -- \
    python3 -u bench.py $args > "$out/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$out/pmc$i.log"; exit 1; }
done
python3 profiles/summarize_r02.py "$out" "$cfg" 3 > "$out/summary.json" || exit 1
echo done
