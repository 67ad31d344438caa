#!/bin/bash
# Round-6 final evidence, second call: the config4 driver command with its
# rocprof stats and PMC passes (scripts/gpu_prof_r5.sh), then the config5 and
# config2 bench lines.   scripts/gpu_r6_final2.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-r6_final2}
mkdir -p "gpurun_out/$OUT"
export TMPDIR=/tmp
bash scripts/gpu_prof_r5.sh "$OUT/prof_config4" config4 1 &&
timeout -k 10 400 python3 -u bench.py --workload config5 --steps 5 --warmup 2 > "gpurun_out/$OUT/bench_c5.json" 2> "gpurun_out/$OUT/bench_c5.err" &&
timeout -k 10 400 python3 -u bench.py --workload config2 > "gpurun_out/$OUT/bench_c2.json" 2> "gpurun_out/$OUT/bench_c2.err" &&
echo done
