#!/bin/bash
# Phase-A cycle stamps for the stamps build and one timing experiment.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps}
EXP=${2:-NOPASS3}
mkdir -p "$OUT"
for wl in config4 config3; do
  for v in stamps exp_$EXP; do
    GS_STAMPS_LIB=libgossip_engine_$v.so timeout -k 10 200 python3 -u scripts/stamps.py $wl > "$OUT/${wl}_$v.txt" 2>&1 || exit 1
  done
done
grep -H "pass\|total" "$OUT"/*.txt | grep -v "phase B\|step"
