#!/bin/bash
# Two quick PMC passes (SQ mix + HBM bytes) for the kernels matching $2.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-pmc}
RE=${2:-k_phase_a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {
  local name=$1
  shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" --output-format csv \
      -d "$OUT/$name" -o run -- python3 -u scripts/prof_driver.py > "$OUT/$name.log" 2>&1
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
echo done
