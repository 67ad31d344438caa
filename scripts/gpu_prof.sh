#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here;
# counter passes run separately, one block set per pass).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-prof}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo done
