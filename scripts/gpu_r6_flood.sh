#!/bin/bash
# Round 6: the dense-frontier floodsub path (k_flood_a): floodsub parity and
# goldens, the 100k closed forms, then the config2 floodsub bench line.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_flood}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread \
    tests/test_golden.py tests/test_parity_gpu.py tests/test_scale_gpu.py -k "floodsub or flood or scale" \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --workload config2 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err" || exit 1
python - "$OUT" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1] + "/bench_config2.json").read().strip().splitlines()[-1])
print("config2", f"{j['value']:.4g}", f"ms/step {j['ms_per_step']:.1f}", j.get("kernel_ms_per_step"), "frac", j.get("roofline", {}).get("frac"))
PY
