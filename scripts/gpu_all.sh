#!/bin/bash
# GPU tests, then the config4 / config3 / config5 benches and the PMC
# calibration program; each step time-limited, chained with &&.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" &&
timeout -k 10 600 python -u bench.py --workload config3 --steps 3 --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 900 python -u bench.py --workload config5 --steps 3 --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
bash scripts/gpu_pmc_calib.sh "${1:-all}_calib" &&
echo done
