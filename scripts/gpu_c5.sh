#!/bin/bash
# config5 (adversarial) bench on one GPU, then the product tests of the
# adversarial scenarios; each step time-limited, chained with &&.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c5}
PEERS=${2:-1000000}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --workload config5 --peers $PEERS --steps 3 --warmup 2 \
    > "$OUT/bench_c5_$PEERS.json" 2> "$OUT/bench_c5_$PEERS.err" &&
echo done
