#!/bin/bash
# Round-6 final evidence on the product library: the GPU suite, smoke(), then
# the config3 / config5 bench lines at the driver's window (config4's driver
# command and its profile: scripts/gpu_prof_r5.sh).  Each step time-limited.
#   scripts/gpu_r6_final.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --workload config3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
echo done
rc=$?
tail -2 "$OUT/pytest_gpu.log"
exit $rc
