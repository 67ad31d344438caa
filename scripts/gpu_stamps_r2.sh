#!/bin/bash
# Phase-A / phase-B cycle stamps (GS_STAMPS builds: make var NAME=stamps
# DEFS=-DGS_STAMPS) at config4 and config3, for the product kernels and the
# NOCAS timing experiment (byte-min CAS loop replaced by a plain store).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps}
mkdir -p "$OUT"
for wl in config3 config4; do
  for v in var_stamps var_exp_NOCAS; do
    GS_STAMPS_LIB=libgossip_engine_$v.so timeout -k 10 200 python3 -u scripts/stamps.py $wl > "$OUT/${wl}_$v.txt" 2>&1 || exit 1
  done
done
echo ok
