"""Debug tool (not a test): step the oracle and the HIP engine one hop at a
time on a scenario and report the first hop at which any readback diverges,
with per-edge details.  Usage: python tests/debug_diverge.py <scenario>"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
sys.path.insert(0, HERE)

import scenarios  # noqa: E402
from pubsub_amd import PRODUCT_LIB  # noqa: E402

ORACLE = os.path.join(os.path.dirname(HERE), "oracle", "_build", "libgossip_oracle.so")


def light(e):
    s = dict(counters=e.counters(), mesh=e.mesh(), fanout=e.fanout(), backoff=e.backoff(),
             scores=e.scores(), bp=e.behaviour_penalty())
    s.update({"ts_" + k: v for k, v in e.topic_stats().items()})
    return s


def main(name, lib=None):
    a, hops = scenarios.SCENARIOS[name](ORACLE)
    b, _ = scenarios.SCENARIOS[name](lib or PRODUCT_LIB)
    for h in range(hops):
        a.step(1)
        b.step(1)
        sa, sb = light(a), light(b)
        bad = scenarios.compare(sa, sb)
        if bad:
            print(f"first divergence after hop {h} (now = {h * 100} ms)")
            for x in bad:
                print("  ", x)
            for k in sa:
                if k == "counters":
                    continue
                x, y = scenarios._bits(sa[k]), scenarios._bits(sb[k])
                diff = np.argwhere(x != y)
                for idx in diff[:6]:
                    idx = tuple(idx)
                    e = idx[-1]
                    u = int(np.searchsorted(a.rowptr, e, side="right") - 1)
                    print(f"   {k}{list(idx)} edge {u}->{a.col[e]}: oracle={sa[k][idx]!r} gpu={sb[k][idx]!r}"
                          f" | mesh o={sa['mesh'][e]} g={sb['mesh'][e]} score o={sa['scores'][e]!r}"
                          f" g={sb['scores'][e]!r}")
            return 1
    print("no divergence over", hops, "hops")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gossipsub_scored", sys.argv[2] if len(sys.argv) > 2 else None))
