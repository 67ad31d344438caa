#!/bin/bash
# Round 6: the whole GPU suite and smoke on the current build (what the driver
# runs at round end).  scripts/gpu_r6_suite.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_suite}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
