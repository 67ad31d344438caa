#!/bin/bash
# Same-box config3 A/B: product library vs variants, twice each (bench.py --lib).
#   scripts/gpu_ab_c3.sh OUT VAR [VAR ...]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab_c3}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
B="go-libp2p-pubsub_amd/build"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 5 --no-cpu-baseline \
      > "$OUT/main_c3_$k.json" 2> "$OUT/main_c3_$k.err" || exit 1
  for v in "$@"; do
    timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 5 --no-cpu-baseline \
        --lib "$B/libgossip_engine_var_$v.so" > "$OUT/${v}_c3_$k.json" 2> "$OUT/${v}_c3_$k.err" || exit 1
  done
done
echo done
