#!/bin/bash
# Round 6: PX under RPC byte accounting and the cut spill, GPU = oracle and
# golden, 1 and 2 ranks.   scripts/gpu_r6_pxacct.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_pxacct}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_px.py tests/test_partition_gpu.py \
    tests/test_abi.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "acct or px or cut or abi" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
