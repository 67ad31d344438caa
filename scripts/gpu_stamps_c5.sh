#!/bin/bash
# Phase A / phase B / heartbeat cycle stamps at config5 (GS_STAMPS build).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps_c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 300 python3 -u scripts/stamps.py config5 61 8 > "$OUT/stamps_config5.txt" 2>&1 &&
echo done
