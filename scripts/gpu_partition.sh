#!/bin/bash
# Partitioned-engine checks on a 1-GPU box: the GPU parity tests (including the
# multi-process partition parity against the oracle), then a 2-rank bench
# rehearsal with the host-staged gloo transport on a reduced graph.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-partition}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
GS_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --peers 100000 \
    > "$OUT/bench_p2.json" 2> "$OUT/bench_p2.err" &&
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --peers 100000 --no-cpu-baseline \
    > "$OUT/bench_p1.json" 2> "$OUT/bench_p1.err" &&
echo done
