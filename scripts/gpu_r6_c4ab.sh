#!/bin/bash
# Round 6: config4 A/B, current build against build/libgossip_engine_var_prev.so, same box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_c4ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in new prev new prev; do
  lib=go-libp2p-pubsub_amd/build/libgossip_engine.so
  [ "$v" = prev ] && lib=go-libp2p-pubsub_amd/build/libgossip_engine_var_prev.so
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --lib "$lib" \
      > "$OUT/bench_c4_$v.json" 2> "$OUT/bench_c4_$v.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms_per_step']; print(sys.argv[2], round(j['value']/1e9,3), 'pa', k['phase_a'], 'pb', k['phase_b'])" "$OUT/bench_c4_$v.json" $v
done
