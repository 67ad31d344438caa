#!/bin/bash
# Round-5 final evidence on the product library: the GPU suite, smoke(), the
# driver's bench command (with its CPU baseline), then config3 / config5 lines
# at the driver's window.  Each step time-limited, chained with &&.
#   scripts/gpu_final_r5.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-final_r5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 400 python -u bench.py --workload config3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 400 python -u bench.py --workload config5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
