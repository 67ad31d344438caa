#!/bin/bash
# RPC accounting parity on the GPU, then config4 bench without and with
# RPC byte accounting (its cost).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-acctb}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "acct" > "$OUT/pytest_acct.txt" 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --rpc-accounting > "$OUT/bench_c4_acct.json" 2> "$OUT/bench_c4_acct.err" &&
echo done
