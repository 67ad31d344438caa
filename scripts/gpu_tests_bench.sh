#!/bin/bash
# GPU tests then a short config4 bench (no CPU baseline), each step time-limited.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-tb}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo done
