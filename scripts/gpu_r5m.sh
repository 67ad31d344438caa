#!/bin/bash
# Heartbeat selection A/B (variants skh1 / skh0), then config3 / config5 PMC
# traffic and the config2 bench lines (scripts/gpu_prof_r5b.sh).
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_ab_quick_r5.sh abq2 skh1 skh0 && bash scripts/gpu_prof_r5b.sh prof_r5b && echo done
