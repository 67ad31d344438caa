#!/bin/bash
# Config3 at steady state: rocprofv3 kernel trace of the default bench (5
# rounds after 2 warm-up rounds), then phase-B cycle stamps at the hops
# after a heartbeat (GS_STAMPS build libgossip_engine_var_stamps.so).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-c3t}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 -u bench.py --workload config3 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
for hops in 51 52 53 54; do
  GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 200 python3 -u scripts/stamps.py config3 $hops > "$OUT/stamps_$hops.txt" 2>&1 || exit 1
done
echo done
