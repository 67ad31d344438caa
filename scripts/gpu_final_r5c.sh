#!/bin/bash
# Final round-5 evidence: suite + smoke + the three bench lines, then the
# config4 driver-command profile (rocprof stats + PMC passes).
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_final_r5.sh "${1:-final_r5c}" && bash scripts/gpu_prof_r5.sh "${2:-prof_r5_c4b}" config4 1 && echo done
