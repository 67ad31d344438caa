#!/bin/bash
# Same-box A/B: the round-3 build (ab_r3/, not committed) against the working
# tree on config4, then the working tree's spam-path parity tests and config5.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline > "$OUT/cur_c4.json" 2> "$OUT/cur_c4.err" &&
(cd ab_r3 && timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline) > "$OUT/r3_c4.json" 2> "$OUT/r3_c4.err" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "spam or adversar or c5 or config5" \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 5 --no-cpu-baseline > "$OUT/cur_c5.json" 2> "$OUT/cur_c5.err" &&
true &&
# phase-B step-2 sub-stamps (make var NAME=pb2 DEFS="-DGS_STAMPS -DGS_STAMPS_PB2")
GS_STAMPS_PB2=1 GS_STAMPS_LIB=libgossip_engine_var_pb2.so timeout -k 10 240 python3 -u scripts/stamps.py config4 \
    > "$OUT/stamps_pb2_config4.txt" 2>&1
