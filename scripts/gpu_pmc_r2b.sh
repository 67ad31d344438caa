#!/bin/bash
# Round-2 final PMC traffic passes (FETCH_SIZE, WRITE_SIZE; one counter per
# run) over every hot kernel at config4, then the config3 bench line.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-pmc_r2b}
ONLY_TRAFFIC=1 bash scripts/gpu_pmc.sh "$TAG" "k_phase_a|k_heartbeat|k_phase_b|k_score|k_refresh|k_fwd" &&
timeout -k 10 600 python -u bench.py --workload config3 --no-cpu-baseline > "gpurun_out/$TAG/bench_c3.json" 2> "gpurun_out/$TAG/bench_c3.err" &&
echo done
