#!/bin/bash
# Round-5 GPU session: the GPU suite (optionally a -k selection), then the
# benches with the driver's window (20 steps after 5 warm-up rounds: config5's
# window starts after hop 50).  Each step time-limited, chained with && so a
# failure stops the session.
#   scripts/gpu_r4.sh OUT [pytest -k expression]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r5}
SEL=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${SEL:+-k "$SEL"} \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python -u bench.py --workload config5 --steps 5 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
if [ -n "$STAMPS" ]; then  # phase-B step-2 sub-stamps (make var NAME=pb2 DEFS="-DGS_STAMPS -DGS_STAMPS_PB2")
  GS_STAMPS_PB2=1 GS_STAMPS_LIB=libgossip_engine_var_pb2.so timeout -k 10 240 python3 -u scripts/stamps.py config4 \
      > "$OUT/stamps_pb2_config4.txt" 2>&1
fi &&
echo done
