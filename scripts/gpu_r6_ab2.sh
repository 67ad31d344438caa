#!/bin/bash
# Round 6: A/B of the current build against the previous commit's
# (build/libgossip_engine_var_prev.so): goldens + parity first, then config4
# and config3 alternately on one box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_ab2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_golden.py tests/test_parity_gpu.py tests/test_midsize_gpu.py tests/test_partition_gpu.py \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for wl in config4 config3; do
for v in new prev new prev; do
  lib=go-libp2p-pubsub_amd/build/libgossip_engine.so
  [ "$v" = prev ] && lib=go-libp2p-pubsub_amd/build/libgossip_engine_var_prev.so
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 3 --lib "$lib" \
      > "$OUT/bench_${wl}_$v.json" 2> "$OUT/bench_${wl}_$v.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms_per_step']; print(sys.argv[2], round(j['value']/1e9,3), k)" "$OUT/bench_${wl}_$v.json" "$wl $v"
done
done
