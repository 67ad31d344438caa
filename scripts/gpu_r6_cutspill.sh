#!/bin/bash
# Round 6: the MaxIHaveLength cut spill (GS_CUTS items in LDS, the rest in the
# rank's cut table): the cut scenarios, GPU = oracle and GPU = golden.
#   scripts/gpu_r6_cutspill.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_cutspill}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_midsize_gpu.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "cut or c3 or spam or adversarial or c5" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
