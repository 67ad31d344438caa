#!/bin/bash
# Round 6: phase A pass stamps at config3, frontier bitmaps vs lists (GS_STAMPS build).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_stamps_c3}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_STAMPS_FRONTIER=bitmaps GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config3 25 4 > "$OUT/stamps_dense.txt" 2>&1 &&
GS_STAMPS_FRONTIER=lists GS_STAMPS_LIB=libgossip_engine_stamps.so timeout -k 10 240 python3 -u scripts/stamps.py config3 25 4 > "$OUT/stamps_lists.txt" 2>&1
rc=$?
cat "$OUT/stamps_dense.txt" "$OUT/stamps_lists.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_frontier_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for m in bitmaps lists; do
  timeout -k 10 300 python -u bench.py --workload config3 --no-cpu-baseline --steps 10 --warmup 3 --frontier $m \
      > "$OUT/bench_c3_$m.json" 2> "$OUT/bench_c3_$m.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(j['value']/1e9,3), j['kernel_ms_per_step'])" "$OUT/bench_c3_$m.json" $m
done
