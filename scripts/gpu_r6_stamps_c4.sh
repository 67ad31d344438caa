#!/bin/bash
# Round 6: phase A / B / heartbeat stamps at config4 (GS_STAMPS build).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_stamps_c4}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 61 8 > "$OUT/stamps.txt" 2>&1
rc=$?
cat "$OUT/stamps.txt"
exit $rc
