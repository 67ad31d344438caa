#!/bin/bash
# Debug: first hop where the GPU diverges from the oracle on a scenario, for
# the product library and any other builds given (go-libp2p-pubsub_amd/build/<lib>).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-div}
NAME=$2
shift 2
mkdir -p "$OUT"
timeout -k 10 300 python -u tests/debug_diverge.py $NAME > "$OUT/product.txt" 2>&1
for lib in "$@"; do
  timeout -k 10 300 python -u tests/debug_diverge.py $NAME go-libp2p-pubsub_amd/build/$lib > "$OUT/$lib.txt" 2>&1
done
echo done
