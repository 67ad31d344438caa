#!/bin/bash
# One GPU-box session: parity tests, smoke, bench lines, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python3 -u scripts/stamps.py > "$OUT/stamps.txt" 2>&1 &&
echo done
