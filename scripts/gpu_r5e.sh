#!/bin/bash
# The GPU suite on the current product library, then a same-box A/B against
# variants (scripts/gpu_ab_r5.sh).   scripts/gpu_r5e.sh OUT VAR...
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-r5e}
shift
mkdir -p "gpurun_out/$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "gpurun_out/$OUT/pytest_gpu.log" 2>&1 &&
bash scripts/gpu_ab_r5.sh "$OUT/ab" "$@"
