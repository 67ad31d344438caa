#!/bin/bash
# config3 and config5 PMC traffic (scripts/gpu_prof_r5.sh without SQ sets),
# then the config2 bench lines.   scripts/gpu_prof_r5b.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-prof_r5b}
mkdir -p "gpurun_out/$OUT"
export TMPDIR=/tmp
bash scripts/gpu_prof_r5.sh "$OUT/config3" config3 0 &&
bash scripts/gpu_prof_r5.sh "$OUT/config5" config5 0 &&
timeout -k 10 400 python3 -u bench.py --workload config2 > "gpurun_out/$OUT/bench_config2.json" 2> "gpurun_out/$OUT/bench_config2.err" &&
timeout -k 10 400 python3 -u bench.py --workload config2_rs100 > "gpurun_out/$OUT/bench_config2_rs100.json" 2> "gpurun_out/$OUT/bench_config2_rs100.err" &&
echo done
