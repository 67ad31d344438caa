#!/bin/bash
# Cycle stamps (GS_STAMPS build: make var NAME=stamps DEFS=-DGS_STAMPS) at
# config4 and config5 past hop 50.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-st}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 \
    > "$OUT/stamps_config4.txt" 2>&1 &&
GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 400 python3 -u scripts/stamps.py config5 56 7 \
    > "$OUT/stamps_config5_h56.txt" 2>&1 &&
echo done
