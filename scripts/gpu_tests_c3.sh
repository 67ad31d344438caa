#!/bin/bash
# GPU tests, then the config3 bench (1M peers, 1 topic), each step time-limited.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-tc3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python -u bench.py --workload config3 --steps 3 --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
echo done
