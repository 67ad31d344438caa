#!/bin/bash
# Round-2 PMC passes: the product build (4 passes), then FETCH/WRITE of the
# phase-A experiment without pass 3 (its pending-count bytes, by difference).
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_pmc.sh pmc_r2 &&
ONLY_TRAFFIC=1 bash scripts/gpu_pmc.sh pmc_r2_nopass3 'k_phase_a' go-libp2p-pubsub_amd/build/libgossip_engine_exp_NOPASS3.so &&
echo done
