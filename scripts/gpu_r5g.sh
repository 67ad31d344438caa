#!/bin/bash
# GPU suite on the product library, same-box A/B against variants
# (scripts/gpu_ab_r5.sh), then config4 phase-A stamps of the product kernels
# and of the variants' stamps builds.   scripts/gpu_r5g.sh OUT VAR...
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-r5g}
shift
mkdir -p "gpurun_out/$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "gpurun_out/$OUT/pytest_gpu.log" 2>&1 &&
bash scripts/gpu_ab_r5.sh "$OUT/ab" "$@" &&
GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 61 8 \
    > "gpurun_out/$OUT/stamps_main.txt" 2>&1 &&
for v in "$@"; do
  if [ -f "go-libp2p-pubsub_amd/build/libgossip_engine_var_stamps_$v.so" ]; then
    GS_STAMPS_LIB=libgossip_engine_var_stamps_$v.so timeout -k 10 240 python3 -u scripts/stamps.py config4 61 8 \
        > "gpurun_out/$OUT/stamps_$v.txt" 2>&1 || exit 1
  fi
done && echo done
