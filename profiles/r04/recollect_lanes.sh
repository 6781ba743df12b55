set -o pipefail
bash profiles/r04/collect.sh gpurun_out/pmc9 C3c C3b C4 PP || exit 1
for c in C3c C3b C4 PP; do cp gpurun_out/pmc9/$c/summary.json profiles/r04/${c}_pmc.json && cp gpurun_out/pmc9/$c/kernel_stats.csv profiles/r04/${c}_kernel_stats.csv || exit 1; done
timeout -k 10 600 python -u bench.py > gpurun_out/bench9.json 2> gpurun_out/bench9.err || { tail -20 gpurun_out/bench9.err; exit 1; }
cat gpurun_out/bench9.json
