#!/bin/bash
# Same-box A/B of build variants on the config4 bench (driver window):
#   scripts/gpu_ab_libs.sh OUT var1 var2 ...  (build/libgossip_engine_var_<v>.so)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline > "$OUT/base.json" 2> "$OUT/base.err" || exit 1
for v in "$@"; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline \
      --lib go-libp2p-pubsub_amd/build/libgossip_engine_var_$v.so > "$OUT/$v.json" 2> "$OUT/$v.err" || exit 1
done
echo done
