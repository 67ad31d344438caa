#!/bin/bash
# Phase-A cycle stamps of the stamps build at config4 and config3.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps}
mkdir -p "$OUT"
for wl in config4 config3; do
  GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 200 python3 -u scripts/stamps.py $wl > "$OUT/${wl}.txt" 2>&1 || exit 1
done
grep -H "pass\|total" "$OUT"/*.txt | grep -v "phase B\|step\|copies"
