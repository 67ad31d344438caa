#!/bin/bash
# Phase-A cycle stamps (GS_STAMPS builds) at config4 and config3, for the
# product kernels and the NOCAS / NOADD+NOCAS timing experiments.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps}
mkdir -p "$OUT"
for wl in config4 config3; do
  for v in stamps exp_NOCAS exp_NOADD+NOCAS; do
    GS_STAMPS_LIB=libgossip_engine_$v.so timeout -k 10 200 python3 -u scripts/stamps.py $wl > "$OUT/${wl}_$v.txt" 2>&1 || exit 1
  done
done
echo ok
