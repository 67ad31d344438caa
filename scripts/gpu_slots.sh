#!/bin/bash
# config4 bench with smaller message windows (slots per topic): capacity A/B.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-slots}
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in ${SLOTS:-256 128 64}; do
  timeout -k 10 400 python -u bench.py --slots $s --no-cpu-baseline > "$OUT/bench_s$s.json" 2> "$OUT/bench_s$s.err" || echo "slots $s failed"
done
echo done
