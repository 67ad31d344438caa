"""Timing-variant check: run golden scenarios on a given build of the product
library (bench.py --lib experiments) and compare their digests with
tests/golden/scenarios.json.  python scripts/golden_lib.py LIB NAME..."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "tests", "golden"))
sys.path.insert(0, os.path.join(HERE, "..", "go-libp2p-pubsub_amd"))

import scenarios  # noqa: E402
from make_golden import digest  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "..", "tests", "golden", "scenarios.json")))
lib = os.path.abspath(sys.argv[1])
bad = 0
for name in sys.argv[2:]:
    ok = digest(scenarios.run(lib, name)) == GOLDEN[name]
    print(name, "ok" if ok else "MISMATCH", flush=True)
    bad += not ok
sys.exit(1 if bad else 0)
