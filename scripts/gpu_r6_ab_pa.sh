#!/bin/bash
# Round 6: phase A list-walk A/B on config4 (same box, one after another):
# the product build, GS_PA_YG (young index from the slot table), GS_PA_YG +
# GS_PA_SS (seen-skip); a correctness pass of each variant on the c4shape
# golden first.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_ab_pa}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in yg ygss; do
  timeout -k 10 300 python -u scripts/golden_lib.py go-libp2p-pubsub_amd/build/libgossip_engine_var_$v.so \
      c4shape c4shape_wide c3shape gossipsub_scored gossipsub_slot_reuse_4t cut_honest_4t push_overflow \
      > "$OUT/golden_$v.log" 2>&1 || { cat "$OUT/golden_$v.log"; exit 1; }
done
for v in base yg ygss base; do
  lib=go-libp2p-pubsub_amd/build/libgossip_engine.so
  [ "$v" != base ] && lib=go-libp2p-pubsub_amd/build/libgossip_engine_var_$v.so
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --lib "$lib" \
      > "$OUT/bench_c4_$v.json" 2> "$OUT/bench_c4_$v.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(j['value']/1e9,3), j['kernel_ms_per_step']['phase_a'])" "$OUT/bench_c4_$v.json" $v
done
echo done
