#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access width (scripts/pmc_calib.hip),
# one counter per rocprofv3 pass.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/build/pmc_calib > "$OUT/plain.txt" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- ./scripts/build/pmc_calib > "$OUT/fetch.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- ./scripts/build/pmc_calib > "$OUT/write.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- ./scripts/build/pmc_calib > "$OUT/trace.log" 2>&1 &&
echo done
