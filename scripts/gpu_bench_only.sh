#!/bin/bash
# Benches only (config4 driver window, config5 past hop 50).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
