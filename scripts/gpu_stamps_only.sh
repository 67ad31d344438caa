#!/bin/bash
# Cycle stamps only (GS_STAMPS build) at config4.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-st}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 > "$OUT/stamps_config4.txt" 2>&1 &&
echo done
