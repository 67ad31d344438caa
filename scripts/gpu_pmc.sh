#!/bin/bash
# PMC counter passes over scripts/prof_driver.py, one counter group per run
# (rocprofv3 does not split passes).  Usage: gpu_pmc.sh TAG [regex]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-pmc}
RE=${2:-k_phase_a|k_heartbeat|k_phase_b|k_score|k_refresh}
LIBARG=${3:+--lib $3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {
  local name=$1
  shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" --output-format csv \
      -d "$OUT/$name" -o run -- python3 -u scripts/prof_driver.py $LIBARG > "$OUT/$name.log" 2>&1
}
[ -n "$ONLY_TRAFFIC" ] || pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES &&
[ -n "$ONLY_TRAFFIC" ] || pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVES &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
echo done
