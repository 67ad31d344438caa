#!/bin/bash
# Adversarial-path check: GPU parity + partition tests, then the config5 bench.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-adv}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 900 python -u bench.py --workload config5 --steps 3 --warmup 2 \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
