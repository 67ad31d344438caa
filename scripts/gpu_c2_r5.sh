#!/bin/bash
# BASELINE config 2 lines: floodsub and randomsub-100 at 100k peers.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c2_r5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --workload config2 > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err" &&
timeout -k 10 400 python3 -u bench.py --workload config2_rs100 > "$OUT/bench_config2_rs100.json" 2> "$OUT/bench_config2_rs100.err" &&
echo done
