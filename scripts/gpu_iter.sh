#!/bin/bash
# One iteration: GPU tests (optionally a pytest -k filter), heartbeat/phase
# cycle stamps at config4 (GS_STAMPS build), a short config4 bench line.
# usage: scripts/gpu_iter.sh OUTNAME [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-iter}
mkdir -p "$OUT"
export TMPDIR=/tmp
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
    > "$OUT/pytest_gpu.log" 2>&1 &&
GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 > "$OUT/stamps_config4.txt" 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo done
