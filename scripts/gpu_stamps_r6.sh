#!/bin/bash
# Round 6: the GS_STAMPS build once at config4 with round 5's failing command
# (stamps.py config4 61 8), after the stamp-index audit (bounds-checked stamp
# macros, phase-B stamps cleared at node entry).  scripts/gpu_stamps_r6.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps_r6}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 61 8 > "$OUT/stamps.txt" 2>&1
rc=$?
cat "$OUT/stamps.txt"
exit $rc
