#!/bin/bash
# Round 6 iteration: the honest GPU parity set, then a same-box A/B of the
# product library against variants (bench.py --lib), config4 and config3.
#   scripts/gpu_r6_ab.sh OUT "TESTS" VAR [VAR ...]   (VAR: libgossip_engine_var_VAR.so)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r6_ab}
TESTS=${2:-tests/test_golden.py tests/test_parity_gpu.py}
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
B="go-libp2p-pubsub_amd/build"
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread $TESTS > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
fi
for wl in config4 config3; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/main_$wl.json" 2> "$OUT/main_$wl.err" || exit 1
  for v in "$@"; do
    timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline \
        --lib "$B/libgossip_engine_var_$v.so" > "$OUT/${v}_$wl.json" 2> "$OUT/${v}_$wl.err" || exit 1
  done
done
python - "$OUT" "$@" <<'PY'
import json, sys
out = sys.argv[1]
for wl in ("config4", "config3"):
    for v in ["main"] + sys.argv[2:]:
        j = json.loads(open(f"{out}/{v}_{wl}.json").read().strip().splitlines()[-1])
        k = j.get("kernel_ms_per_step", {})
        print(wl, v, f"{j['value']:.4g}", f"ms/step {j['ms_per_step']:.1f}",
              " ".join(f"{a}={b:.1f}" for a, b in k.items()), "frac", j.get("roofline", {}).get("frac"))
PY
