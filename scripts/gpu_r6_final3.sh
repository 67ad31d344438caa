#!/bin/bash
# Round-6 closing bench lines on the current build: config3 and config5.
#   scripts/gpu_r6_final3.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_final3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --workload config3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 400 python3 -u bench.py --workload config5 --steps 5 --warmup 2 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
