#!/bin/bash
# peertx occupancy (GS_STAMPS build) at config5 and config4, and a kernel
# trace of the config5 bench (k_ptx_rebuild's share).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ptx}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/ptx_occupancy.py config5 70 > "$OUT/ptx_config5.txt" 2>&1 &&
timeout -k 10 200 python3 -u scripts/ptx_occupancy.py config4 40 > "$OUT/ptx_config4.txt" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o c5 -- python3 -u bench.py --workload config5 \
    --steps 3 --warmup 5 --no-cpu-baseline > "$OUT/bench_c5_prof.json" 2> "$OUT/bench_c5_prof.err" &&
echo done
