#!/bin/bash
# Same-box A/B, benches only: config4 and config3 (main, variants, main again),
# then config5 for the variants.   scripts/gpu_ab_quick_r5.sh OUT VAR...
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-abq}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
B="go-libp2p-pubsub_amd/build"
run() {  # name lib workload
  local lib=""
  [ "$2" = main ] || lib="--lib $B/libgossip_engine_var_$2.so"
  timeout -k 10 300 python -u bench.py --workload "$3" --steps 20 --warmup 5 --no-cpu-baseline $lib \
      > "$OUT/$1.json" 2> "$OUT/$1.err"
}
for wl in config4 config3 config5; do
  run "main_$wl" main $wl || exit 1
  for v in "$@"; do run "${v}_$wl" "$v" $wl || exit 1; done
done
run main_config4_again main config4 && echo done
