#!/bin/bash
# Quick check after a kernel change: gpu parity tests, then one bench line
# (no CPU baseline).  Each GPU step time-limited; stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
