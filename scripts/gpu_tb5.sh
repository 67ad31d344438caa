#!/bin/bash
# GPU tests, then the config4 and config3 benches at bench.py's default
# 5 timed rounds after 2 warm-up rounds (steady-state gossip load).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-tb5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" &&
timeout -k 10 600 python -u bench.py --workload config3 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
echo done
