#!/bin/bash
# config3: bench (driver window) and phase-B step-2 sub-stamps at a serve hop.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c3}
mkdir -p "$OUT"
export TMPDIR=/tmp
true && \
GS_STAMPS_PB2=1 GS_STAMPS_LIB=libgossip_engine_var_pb2.so timeout -k 10 300 python3 -u scripts/stamps.py config3 53 7 \
    > "$OUT/stamps_pb2_config3_h53.txt" 2>&1 &&
GS_STAMPS_PB2=1 GS_STAMPS_LIB=libgossip_engine_var_pb2.so timeout -k 10 300 python3 -u scripts/stamps.py config3 54 7 \
    > "$OUT/stamps_pb2_config3_h54.txt" 2>&1 &&
echo done
