#!/bin/bash
# Round 6: phase A's dense pass 1 for one-topic gossipsub (k_phase_a DENSE):
# both frontier modes against the goldens, the golden / trace suites (incl. the
# peertx spill runs), then config3 bench lines with bitmaps and with lists.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_dense}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_frontier_gpu.py tests/test_golden.py tests/test_trace.py tests/test_trace_rpc.py \
    > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --workload config3 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 400 python -u bench.py --workload config3 --no-cpu-baseline --steps 10 --warmup 3 --frontier lists > "$OUT/bench_c3_lists.json" 2> "$OUT/bench_c3_lists.err" &&
echo done
