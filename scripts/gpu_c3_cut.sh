#!/bin/bash
# GPU suite, then config3 at bench.py's defaults under a rocprofv3 kernel trace
# (the MaxIHaveLength cut rounds), then config4 at defaults.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c3cut}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 -u bench.py --workload config3 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" &&
echo done
