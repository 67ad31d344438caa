#!/bin/bash
# Round 6: the promise table sized by its liveness bound past 512 entries.
# The previous build (cap 512) must refuse promise_flood_long with E_PROMISES;
# the current one must equal the oracle and the golden.   scripts/gpu_r6_prom.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_prom}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u - > "$OUT/prev_lib.txt" 2>&1 <<'PY'
import sys
sys.path[:0] = ["tests", "go-libp2p-pubsub_amd"]
import scenarios
try:
    e, hops = scenarios.SCENARIOS["promise_flood_long"]("go-libp2p-pubsub_amd/build/libgossip_engine_var_prev.so")
    e.step(hops)
    print("previous build: no error")
except Exception as ex:
    print("previous build:", type(ex).__name__, ex)
PY
cat "$OUT/prev_lib.txt"
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "promise" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
