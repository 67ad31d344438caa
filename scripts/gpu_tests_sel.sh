#!/bin/bash
# Selected GPU tests (pytest -k / file arguments), time-limited.
# usage: scripts/gpu_tests_sel.sh OUTNAME PYTEST_ARGS...
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-sel}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1 &&
echo done
