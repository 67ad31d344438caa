#!/bin/bash
# A/B timing of phase-A variants on one box: GPU parity tests with the product
# library, then the config4 bench with it and with each listed variant
# (build/libgossip_engine_<name>.so swapped in place of the product library).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
B=go-libp2p-pubsub_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$OUT/bench_product.json" 2> "$OUT/bench_product.err" || exit 1
cp $B/libgossip_engine.so /tmp/product.so
for v in "$@"; do
  cp $B/libgossip_engine_$v.so $B/libgossip_engine.so &&
  timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || exit 1
done
cp /tmp/product.so $B/libgossip_engine.so
echo done
