#!/bin/bash
# Kernel-time A/B of timing-experiment builds (results not exact) vs the product.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-expb}
shift
mkdir -p "$OUT"
for wl in config4 config3; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/${wl}_product.json" 2>"$OUT/err.txt" || exit 1
  for lib in "$@"; do
    timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline \
      --lib go-libp2p-pubsub_amd/build/$lib > "$OUT/${wl}_$lib.json" 2>>"$OUT/err.txt" || exit 1
  done
done
for f in "$OUT"/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e9,3), d['kernel_ms_per_step'])"; done
