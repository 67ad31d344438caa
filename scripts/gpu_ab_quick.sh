#!/bin/bash
# Bench-only A/B on one box: the product library, then each listed variant
# (build/libgossip_engine_var_<name>.so swapped in), config4, 3 rounds after 1.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-abq}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
B=go-libp2p-pubsub_amd/build
cp $B/libgossip_engine.so /tmp/product.so
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_product.json" 2> "$OUT/bench_product.err" || exit 1
for v in "$@"; do
  cp $B/libgossip_engine_var_$v.so $B/libgossip_engine.so &&
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { cp /tmp/product.so $B/libgossip_engine.so; exit 1; }
done
cp /tmp/product.so $B/libgossip_engine.so
echo done
