#!/bin/bash
# Round-5 evidence for one workload: the driver's bench command, rocprofv3
# --kernel-trace --stats of the same command, then PMC passes (one counter set
# per run; FETCH_SIZE / WRITE_SIZE always, the SQ sets with SQ=1).  Each step
# time-limited, chained with &&.   scripts/gpu_prof_r5.sh OUT WORKLOAD [SQ]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-prof_r5}
WL=${2:-config4}
SQ=${3:-0}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --workload $WL"
RE='k_phase_a|k_heartbeat|k_phase_b|k_score|k_refresh|k_fwd|k_push|k_ptx_rebuild|k_hb_pre'
pass() {
  local name=$1
  shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" --output-format csv \
      -d "$OUT/$name" -o run -- python3 -u $CMD --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err"
}
timeout -k 10 400 python3 -u $CMD > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 -u $CMD --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" &&
pass fetch FETCH_SIZE && pass write WRITE_SIZE &&
{ [ "$SQ" = 0 ] || {
  pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES &&
  pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVES; }; } &&
echo done
