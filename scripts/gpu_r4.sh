#!/bin/bash
# Round-4 GPU session: the GPU suite (optionally a -k selection), then the
# config5 bench with its window after hop 50 (5 warm-up rounds).  Each step
# time-limited, chained with && so a failure stops the session.
#   scripts/gpu_r4.sh OUT [pytest -k expression]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r4}
SEL=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${SEL:+-k "$SEL"} \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
