#!/bin/bash
# Bench lines of the other workloads (config3 steady state, config4's subnet
# variant) and a kernel trace of the config5 bench for the timing cross-check.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-mb}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload config3 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run -- \
    python3 -u bench.py --workload config5 --steps 5 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c5_prof.json" 2> "$OUT/bench_c5_prof.err" &&
echo done
