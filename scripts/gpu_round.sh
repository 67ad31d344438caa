#!/bin/bash
# Round evidence in one GPU session: gpu tests, smoke, bench line, rocprofv3
# kernel-trace --stats of the same bench command, then the config3 and config5
# bench lines.  Each step time-limited, chained with && so a failure stops the
# session.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-round}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" &&
timeout -k 10 600 python -u bench.py --workload config3 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 600 python -u bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo done
