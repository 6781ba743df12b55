#!/bin/bash
# One bench line per BASELINE config (C1..C5 plus the C3 variants) with its CPU baseline, on one MI355X.
# usage: profiles/all_configs.sh <outdir>     (run on the GPU box via gpurun)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=$1
mkdir -p "$out"
for c in C1 C2 C3 C3b C3c C4 C5; do
  steps=5; [ "$c" == "C3c" ] && steps=2
  timeout -k 10 240 python3 -u bench.py --config $c --steps $steps --warmup 1 > "$out/$c.json" 2> "$out/$c.err" || { echo "$c failed"; tail -5 "$out/$c.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$out/$c.json'));print('$c', d['value'], d['ms_per_step'], (d['cpu_baseline'] or {}).get('value'))"
done
echo done
