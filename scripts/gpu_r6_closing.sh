#!/bin/bash
# Round 6 closing check: the whole GPU suite, smoke, and the config4 driver
# bench on the current build.   scripts/gpu_r6_closing.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_closing}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
rc=$?
tail -2 "$OUT/pytest_gpu.log"
exit $rc
