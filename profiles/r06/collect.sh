#!/bin/bash
# Round-6 evidence per config (on the GPU box via gpurun), one config after another:
#   1. rocprofv3 --kernel-trace --stats of `bench.py --config <cfg>` (per-kernel durations + stats CSV)
#   2. separate --pmc passes FETCH_SIZE | WRITE_SIZE (MI355X_MICROARCH.md §HBM: one TCC group per pass)
#   3. profiles/r06/summarize.py -> <out>/<cfg>/summary.json (per engine mark: avg us and HBM bytes per push),
#      stamped with the kernel-source hash bench.py checks before it uses the traffic figure
# The summaries time the headline alone (the node stage runs the same engine kernels, which would be counted twice);
# for C5 one more --pmc pass runs the whole bench line WITH its whole-node stage (G = 1 and the G = 2 exchange) and its
# log is kept (r05 ran its counter passes with --c5-node-steps 0 after a crash there).
# usage: profiles/r06/collect.sh <outdir> <cfg> [<cfg> ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
for cfg in "$@"; do
  d="$out/$cfg"
  mkdir -p "$d"
  args="--config $cfg --steps 2 --warmup 1 --no-cpu --other-configs= --stream-configs= --c5-node-steps 0"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -o run -- \
    python3 -u bench.py $args > "$d/trace.log" 2>&1 || { echo "$cfg trace failed"; tail -5 "$d/trace.log"; exit 1; }
  i=0
  for g in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $g --output-format csv -d "$d/pmc$i" -o run -- \
      python3 -u bench.py $args > "$d/pmc$i.log" 2>&1 || { echo "$cfg pmc pass $i failed"; tail -5 "$d/pmc$i.log"; exit 1; }
  done
  if [ "$cfg" == "C5" ]; then
    timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d/pmc_node" -o run -- \
      python3 -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu --other-configs= --stream-configs= --c5-node-steps 1 \
      --node-shards 2 > "$d/pmc_node.log" 2>&1 || { echo "C5 pmc pass with the whole-node stage failed"; tail -5 "$d/pmc_node.log"; exit 1; }
    rm -rf "$d/pmc_node"
  fi
  python3 profiles/r06/summarize.py "$d" "$cfg" > "$d/summary.json" || exit 1
  f=$(find "$d/trace" -name "run_kernel_stats.csv" | head -1)
  cp "$f" "$d/kernel_stats.csv"
  echo "$cfg done"
done
