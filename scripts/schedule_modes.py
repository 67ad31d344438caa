"""Runs every parity scenario on the oracle twice — the engine's canonical
schedule and the reference's per-RPC order with live scores
(gs_oracle_reference_order) — and prints how far apart the results are.
The table goes into DESIGN.md §3; tests/test_oracle_schedule.py pins it."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import scenarios  # noqa: E402

ORACLE = os.path.join(REPO, "oracle", "_build", "libgossip_oracle.so")


def run(name, ref):
    e, hops = scenarios.SCENARIOS[name](ORACLE)
    if ref:
        rc = e.lib.gs_oracle_reference_order(e.h, C.c_int32(ref))
        assert rc == 0
    e.step(hops)
    return scenarios.snapshot(e, getattr(e, "snapshot_ids", range(e.n_published))), e


def distance(a, b):
    out = {}
    dh = df = n = 0
    for (h1, f1), (h2, f2) in zip(a["deliv"], b["deliv"]):
        ok = (h1 >= 0) | (h2 >= 0)
        n += int(ok.sum())
        dh += int((h1 != h2)[ok].sum())
        df += int(((f1 != f2) & (h1 == h2))[ok].sum())
    out["deliveries"] = (a["counters"]["deliveries"], b["counters"]["deliveries"])
    out["first_hop_diff"] = dh / max(1, n)
    out["first_from_diff"] = df / max(1, n)
    m1, m2 = a["mesh"], b["mesh"]
    out["mesh_diff"] = float(np.mean(m1 != m2))
    s1, s2 = a["scores"], b["scores"]
    out["score_diff"] = float(np.mean(s1.view(np.uint64) != s2.view(np.uint64)))
    out["counters_diff"] = {k: (a["counters"][k], b["counters"][k]) for k in a["counters"]
                            if a["counters"][k] != b["counters"][k]}
    return out


if __name__ == "__main__":
    names = sys.argv[1:] or [n for n in scenarios.SCENARIOS if n not in scenarios.HEAVY]
    for name in names:
        a, _ = run(name, False)
        b, _ = run(name, 1)
        c, _ = run(name, 2)
        print(name, "per-RPC:", distance(a, b), flush=True)
        print(name, "live-score:", distance(a, c), flush=True)
