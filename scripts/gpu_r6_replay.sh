#!/bin/bash
# Round 6: the full-size per-host replay tests (N1) on the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_replay}
mkdir -p "$OUT"
shift
timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 1000 --timeout-method thread tests/test_fullsize_gpu.py \
    -k "${1:-replay}" > "$OUT/replay.log" 2>&1
rc=$?
tail -5 "$OUT/replay.log"
exit $rc
