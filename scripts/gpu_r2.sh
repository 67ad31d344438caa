#!/bin/bash
# Round-2 GPU session: all gpu tests (no -x: see every mismatch), smoke, bench.
# Each GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo done
