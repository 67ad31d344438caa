#!/bin/bash
# GPU tests, then config4 and config5 bench lines.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-iter2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
