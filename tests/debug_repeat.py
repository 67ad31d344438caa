"""Debug tool (not a test): run a scenario on the product library several
times in one call and print the counters, to tell a race from a logic error.
Usage: python tests/debug_repeat.py <scenario> [repeats]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
sys.path.insert(0, HERE)

import scenarios  # noqa: E402
from pubsub_amd import PRODUCT_LIB  # noqa: E402

name = sys.argv[1]
for r in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    e, hops = scenarios.SCENARIOS[name](PRODUCT_LIB)
    e.step(hops)
    print(r, "one call", e.counters(), flush=True)
    e, hops = scenarios.SCENARIOS[name](PRODUCT_LIB)
    for h in range(hops):
        e.step(1)
    print(r, "stepwise", e.counters(), flush=True)
