#!/bin/bash
# Per-rank footprint of the partitioned engine (scripts/mem_probe.py): config5
# rank 0 of 8 at 1M peers, then at BASELINE's 10M.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-memprobe}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/mem_probe.py --workload config5 --peers 1000000 --world 8 \
    > "$OUT/c5_1m_w8.json" 2> "$OUT/c5_1m_w8.err" &&
timeout -k 10 1050 python -u scripts/mem_probe.py --workload config5 --peers 10000000 --world 8 \
    > "$OUT/c5_10m_w8.json" 2> "$OUT/c5_10m_w8.err" &&
cat "$OUT"/*.json
