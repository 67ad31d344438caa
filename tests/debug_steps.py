"""Debug tool (not a test): step a scenario on the product library one hop at
a time, printing each hop, to locate a hop that does not finish.
Usage: python tests/debug_steps.py <scenario>"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
sys.path.insert(0, HERE)

import scenarios  # noqa: E402
from pubsub_amd import PRODUCT_LIB  # noqa: E402

e, hops = scenarios.SCENARIOS[sys.argv[1]](PRODUCT_LIB)
for h in range(hops):
    t0 = time.time()
    e.step(1)
    e.sync()
    print(h, round(time.time() - t0, 3), flush=True)
print("done", e.counters())
