#!/bin/bash
# Full-size (config4, 1M peers) rehearsal of the partitioned bench path on a
# 1-GPU box: 2 ranks share the GPU, host-staged gloo transport.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-rehearse}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_DIST_BACKEND=gloo timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 \
    > "$OUT/bench_p2.json" 2> "$OUT/bench_p2.err" &&
echo done
