#!/bin/bash
# Round-5 evidence per config (on the GPU box via gpurun), one config after another:
#   1. rocprofv3 --kernel-trace --stats of `bench.py --config <cfg>` (per-kernel durations + stats CSV)
#   2. separate --pmc passes FETCH_SIZE | WRITE_SIZE (MI355X_MICROARCH.md §HBM: one TCC group per pass)
#   3. profiles/r05/summarize.py -> <out>/<cfg>/summary.json (per engine mark: avg us and HBM bytes per push),
#      stamped with the kernel-source hash bench.py checks before it uses the traffic figure
# usage: profiles/r05/collect.sh <outdir> <cfg> [<cfg> ...]   (copy <outdir>/<cfg>/summary.json to profiles/r05/<cfg>_pmc.json)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
for cfg in "$@"; do
  d="$out/$cfg"
  mkdir -p "$d"
  args="--config $cfg --steps 2 --warmup 1 --no-cpu --other-configs= --c5-node-steps 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -o run -- \
    python3 -u bench.py $args > "$d/trace.log" 2>&1 || { echo "$cfg trace failed"; tail -5 "$d/trace.log"; exit 1; }
  i=0
  for g in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d "$d/pmc$i" -o run -- \
      python3 -u bench.py $args > "$d/pmc$i.log" 2>&1 || { echo "$cfg pmc pass $i failed"; tail -5 "$d/pmc$i.log"; exit 1; }
  done
  python3 profiles/r05/summarize.py "$d" "$cfg" > "$d/summary.json" || exit 1
  f=$(find "$d/trace" -name "run_kernel_stats.csv" | head -1)
  cp "$f" "$d/kernel_stats.csv"
  echo "$cfg done"
done
