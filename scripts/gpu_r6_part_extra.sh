#!/bin/bash
# Round 6: the new partitioned cases (promise table, PX accounting at 3 ranks).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_part_extra}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_partition_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "promise_flood_long or acct_px or cut_spill" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log"
exit $rc
