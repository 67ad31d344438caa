#!/bin/bash
# Config 5 (adversarial mix) at 2M peers on one GPU: capacity check + bench line.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c5_2m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --workload config5 --peers 2000000 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_c5_2m.json" 2> "$OUT/bench_c5_2m.err" &&
echo done
