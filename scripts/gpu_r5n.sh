#!/bin/bash
# GPU suite, then config5 with and without the recorded drop copies
# (GS_DEBUG_NO_DROPBUF), then config4 / config3 lines.   scripts/gpu_r5n.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r5n}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
$B --workload config5 > "$OUT/c5_dropbuf.json" 2> "$OUT/c5_dropbuf.err" &&
GS_DEBUG_NO_DROPBUF=1 $B --workload config5 > "$OUT/c5_walk.json" 2> "$OUT/c5_walk.err" &&
$B --workload config5 > "$OUT/c5_dropbuf_again.json" 2> "$OUT/c5_dropbuf_again.err" &&
$B --workload config4 > "$OUT/c4.json" 2> "$OUT/c4.err" &&
$B --workload config3 > "$OUT/c3.json" 2> "$OUT/c3.err" &&
echo done
