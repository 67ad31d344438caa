#!/bin/bash
# Round 6: config4 driver bench on the current build (regression check), twice.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_c4check}
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_c4_$k.json" 2> "$OUT/bench_c4_$k.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(j['value']/1e9,3), j['kernel_ms_per_step'])" "$OUT/bench_c4_$k.json"
done
