"""Debug tool (not a test): run a scenario with every node traced on the
oracle and the HIP engine, hop by hop, and print the first hop whose event
streams differ, with the differing events of that hop.
Usage: python tests/debug_trace_diff.py <scenario> [max_hops]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
sys.path.insert(0, HERE)

import scenarios  # noqa: E402
from pubsub_amd import PRODUCT_LIB, WithEventTracer  # noqa: E402

ORACLE = os.path.join(os.path.dirname(HERE), "oracle", "_build", "libgossip_oracle.so")


def main(name, max_hops=10 ** 9):
    probe, hops = scenarios.SCENARIOS[name](ORACLE)
    nodes = list(range(probe.N))
    a, _ = scenarios.SCENARIOS[name](ORACLE, (WithEventTracer(nodes),))
    b, _ = scenarios.SCENARIOS[name](PRODUCT_LIB, (WithEventTracer(nodes),))
    alla, allb = [], []
    for h in range(min(hops, max_hops)):
        a.step(1)
        b.step(1)
        ea, eb = a.trace_events(), b.trace_events()
        alla.append(ea)
        allb.append(eb)
        ca, cb = a.counters(), b.counters()
        if len(ea) == len(eb) and (ea == eb).all() and ca == cb:
            continue
        print(f"hop {h}: {len(ea)} oracle events, {len(eb)} gpu events")
        print({k: (ca[k], cb[k]) for k in ca if ca[k] != cb[k]})
        sa = {tuple(r) for r in ea.tolist()}
        sb = {tuple(r) for r in eb.tolist()}
        print("fields:", ea.dtype.names)
        for r in sorted(sa - sb)[:40]:
            print("  oracle only:", r)
        for r in sorted(sb - sa)[:40]:
            print("  gpu only:   ", r)
        fa, fb = np.concatenate(alla), np.concatenate(allb)
        for r in sorted(sa ^ sb)[:4]:
            node, msg = r[3], r[1]
            print(f"-- node {node} msg {msg}: oracle / gpu")
            for x in fa[(fa["node"] == node) & (fa["msg"] == msg)].tolist():
                print("   o", x)
            for x in fb[(fb["node"] == node) & (fb["msg"] == msg)].tolist():
                print("   g", x)
        node = sorted(sa ^ sb)[0][3]
        print(f"-- all hop-{h} events of node {node} (oracle):")
        for x in ea[ea["node"] == node].tolist():
            print("   o", x)
        print(f"-- hop-{h} events of node {node} that differ in order/content (gpu):")
        for x in eb[eb["node"] == node].tolist():
            print("   g", x)
        return 1
    print("no divergence")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10 ** 9))
