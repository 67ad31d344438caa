#!/bin/bash
# Same-box A/B of the product library against timing variants (bench.py --lib),
# config4 at the driver's window; then the variants' config3 / config5 lines.
#   scripts/gpu_ab_r5.sh OUT VAR [VAR ...]   (VAR: libgossip_engine_var_VAR.so)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab_r5}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
B="go-libp2p-pubsub_amd/build"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/main_c4.json" 2> "$OUT/main_c4.err" &&
for v in "$@"; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --lib "$B/libgossip_engine_var_$v.so" \
      > "$OUT/${v}_c4.json" 2> "$OUT/${v}_c4.err" || exit 1
done &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/main_c4_again.json" 2> "$OUT/main_c4_again.err" &&
timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/main_c3.json" 2> "$OUT/main_c3.err" &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/main_c5.json" 2> "$OUT/main_c5.err" &&
for v in "$@"; do
  timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 5 --no-cpu-baseline \
      --lib "$B/libgossip_engine_var_$v.so" > "$OUT/${v}_c5.json" 2> "$OUT/${v}_c5.err" || exit 1
  timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 5 --no-cpu-baseline \
      --lib "$B/libgossip_engine_var_$v.so" > "$OUT/${v}_c3.json" 2> "$OUT/${v}_c3.err" || exit 1
done &&
echo done
