#!/bin/bash
# Round 6: the heartbeat's steady-topic fast path: parity (goldens, live
# oracle, traces, mid-size incl. c4steady), then config4 A/B against the
# previous build (build/libgossip_engine_var_headhb.so) on the same box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_hb}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_golden.py tests/test_parity_gpu.py tests/test_trace.py tests/test_trace_rpc.py tests/test_midsize_gpu.py \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in new head new head; do
  lib=go-libp2p-pubsub_amd/build/libgossip_engine.so
  [ "$v" = head ] && lib=go-libp2p-pubsub_amd/build/libgossip_engine_var_headhb.so
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --lib "$lib" \
      > "$OUT/bench_c4_$v.json" 2> "$OUT/bench_c4_$v.err" || exit 1
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms_per_step']; print(sys.argv[2], round(j['value']/1e9,3), 'hb', k['heartbeat'], 'pa', k['phase_a'])" "$OUT/bench_c4_$v.json" $v
done
