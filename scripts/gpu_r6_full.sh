#!/bin/bash
# Round 6: the whole GPU suite on the current build, smoke, and the config4 /
# config3 bench lines.  Each step time-limited, chained with &&.
#   scripts/gpu_r6_full.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_full}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 400 python -u bench.py --workload config3 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
echo done
