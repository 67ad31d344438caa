"""Debug tool (not a test): per-edge RPC accounting differences between the
oracle and the product on a scenario.  Usage: python tests/debug_acct.py <name>"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
sys.path.insert(0, HERE)

import scenarios  # noqa: E402
from pubsub_amd import PRODUCT_LIB  # noqa: E402

ORACLE = os.path.join(os.path.dirname(HERE), "oracle", "_build", "libgossip_oracle.so")
name = sys.argv[1]
res = {}
for tag, lib in (("oracle", ORACLE), ("gpu", PRODUCT_LIB)):
    e, hops = scenarios.SCENARIOS[name](lib)
    rows = []
    for h in range(hops):
        e.step(1)
        rows.append(e.rpc_bytes())
    res[tag] = (e, rows)
eo, ro = res["oracle"]
eg, rg = res["gpu"]
rowptr = eo.rowptr
src = np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr))
for h, ((bo, no), (bg, ng)) in enumerate(zip(ro, rg)):
    bad = np.flatnonzero((bo != bg) | (no != ng))
    if len(bad):
        print("first divergence at hop", h)
        for k in bad[:10]:
            print(f"  edge {k}: {src[k]} -> {eo.col[k]}  oracle bytes {bo[k]} rpcs {no[k]}  gpu bytes {bg[k]} rpcs {ng[k]}"
                  f"  (hop before: oracle {ro[h-1][0][k] if h else 0}/{ro[h-1][1][k] if h else 0},"
                  f" gpu {rg[h-1][0][k] if h else 0}/{rg[h-1][1][k] if h else 0})")
        break
else:
    print("no divergence")
