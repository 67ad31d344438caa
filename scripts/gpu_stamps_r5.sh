#!/bin/bash
# Round-5 phase-A cycle stamps (GS_STAMPS builds, scripts/stamps.py) at config4's
# benchmarked window: the product kernels' stamps build, then the timing
# experiments (NOCAS: no byte-min CAS; NOADD+NOCAS: no LDS counter adds either;
# their results are not exact, stamps only).  scripts/gpu_stamps_r5.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-stamps_r5}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in stamps exp_NOCAS exp_NOADD+NOCAS; do
  GS_STAMPS_LIB=libgossip_engine_$v.so timeout -k 10 240 python3 -u scripts/stamps.py config4 61 8 \
      > "$OUT/$v.txt" 2>&1 || exit 1
done
echo done
