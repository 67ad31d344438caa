#!/bin/bash
# Config3 phase-B cycle stamps at the hops after the heartbeats of rounds 5-7
# (GS_STAMPS build libgossip_engine_var_stamps.so; bench.py's 8-round schedule).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c3s}
mkdir -p "$OUT"
for hops in 42 52 62; do
  GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 200 python3 -u scripts/stamps.py config3 $hops 8 > "$OUT/stamps_$hops.txt" 2>&1 || exit 1
done
echo done
