#!/bin/bash
# Cycle stamps of config5 (adversarial) at 1M peers: phase A / B / heartbeat.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c5st}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 400 python3 -u scripts/stamps.py config5 36 5 \
    > "$OUT/stamps_config5_h36.txt" 2>&1 &&
GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 400 python3 -u scripts/stamps.py config5 33 5 \
    > "$OUT/stamps_config5_h33.txt" 2>&1 &&
echo done
