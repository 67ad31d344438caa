#!/bin/bash
# Round 6: the dense pass 1 without register spills: frontier-mode parity, then
# config3 with bitmaps and with lists on the same box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_dense2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_frontier_gpu.py > "$OUT/pytest.log" 2>&1 &&
for m in auto lists; do
  timeout -k 10 300 python -u bench.py --workload config3 --no-cpu-baseline --steps 10 --warmup 3 --frontier $m \
      > "$OUT/bench_c3_$m.json" 2> "$OUT/bench_c3_$m.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(j['value']/1e9,3), j['kernel_ms_per_step'])" "$OUT/bench_c3_$m.json" $m
done
