#!/bin/bash
# Adversarial-model GPU tests, then the config5 bench line.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-adv}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    -k "spam or adversarial or c5 or sinkhole or squat or acct" > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python -u bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
