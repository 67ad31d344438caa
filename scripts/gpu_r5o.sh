#!/bin/bash
# GPU suite on the product library, then the benches-only A/B against variants.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-r5o}
shift
mkdir -p "gpurun_out/$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "gpurun_out/$OUT/pytest_gpu.log" 2>&1 &&
bash scripts/gpu_ab_quick_r5.sh "$OUT/ab" "$@" && echo done
