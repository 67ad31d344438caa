#!/bin/bash
# Round 6: heartbeat occupancy A/B (GS_WPE_HB=5 vs the default 6) on config4.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_ab3}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in new hb5 new hb5; do
  lib=go-libp2p-pubsub_amd/build/libgossip_engine.so
  [ "$v" != new ] && lib=go-libp2p-pubsub_amd/build/libgossip_engine_var_$v.so
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --lib "$lib" \
      > "$OUT/bench_c4_$v.json" 2> "$OUT/bench_c4_$v.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms_per_step']; print(sys.argv[2], round(j['value']/1e9,3), 'hb', k['heartbeat'], 'push', k['push'])" "$OUT/bench_c4_$v.json" $v
done
