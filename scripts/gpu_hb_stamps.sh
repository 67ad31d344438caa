#!/bin/bash
# Heartbeat / phase-A / phase-B cycle stamps (GS_STAMPS build:
# make var NAME=stamps DEFS=-DGS_STAMPS) at config4 and config3.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-hbstamps}
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in config4 config3; do
  GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py $wl > "$OUT/${wl}.txt" 2>&1 || exit 1
done
echo ok
