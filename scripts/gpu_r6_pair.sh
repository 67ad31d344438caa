#!/bin/bash
# Round 6: message-id keys from both halves of a Philox block + randomsub on a
# partitioned engine.  Goldens / parity / mid-size / partition tests, then the
# config3 and config4 bench lines.  Each step time-limited, chained with &&.
#   scripts/gpu_r6_pair.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_pair}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_golden.py tests/test_parity_gpu.py tests/test_midsize_gpu.py tests/test_partition_gpu.py \
    tests/test_trace.py tests/test_trace_rpc.py > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --workload config3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 400 python -u bench.py > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" &&
echo done
