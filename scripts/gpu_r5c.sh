#!/bin/bash
# Round-5 check after the occupancy fixes: the parity cases the round-5
# changes touch, then config4 / config5 / config3 benches at the driver's
# window, then phase-A stamps (snapshot-built GS_STAMPS variant).  Each step
# time-limited and chained with &&.   scripts/gpu_r5c.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r5c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "golden or midsize or parity or (partitioned and (c4shape or cut_honest or push_overflow or adversarial))" \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
if [ -f go-libp2p-pubsub_amd/build/libgossip_engine_var_stamps.so ]; then
  GS_STAMPS_LIB=libgossip_engine_var_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config4 61 8 \
      > "$OUT/stamps_config4.txt" 2>&1
fi &&
echo done
