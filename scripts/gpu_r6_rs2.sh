#!/bin/bash
# Round 6: randomsub targets drawn two messages per wave step (rs_select2):
# randomsub parity (GPU = oracle, goldens, partitioned), then config2_rs100
# A/B against the previous build on the same box.   scripts/gpu_r6_rs2.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_rs2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_partition_gpu.py \
    tests/test_fullsize_gpu.py tests/test_scale_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "randomsub or rs" > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for v in new prev new prev; do
  lib=go-libp2p-pubsub_amd/build/libgossip_engine.so
  [ "$v" = prev ] && lib=go-libp2p-pubsub_amd/build/libgossip_engine_var_prev.so
  timeout -k 10 300 python -u bench.py --workload config2_rs100 --no-cpu-baseline --steps 3 --warmup 1 --lib "$lib" \
      > "$OUT/bench_rs_$v.json" 2> "$OUT/bench_rs_$v.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(j['value']/1e9,3), j['kernel_ms_per_step'])" "$OUT/bench_rs_$v.json" $v
done
