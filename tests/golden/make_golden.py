"""Generates tests/golden/scenarios.json: for every parity scenario, the
oracle's counters and a SHA-256 digest of every readback array (float64 on
their bit patterns).  The oracle is the CPU restatement pinned by the
reference's known-answer tests; these vectors pin the
simulator-level results so any change to the oracle or the engine that alters
a single bit is caught.  Usage: python tests/golden/make_golden.py [name ...]"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REPO = os.path.dirname(TESTS)
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, TESTS)

import scenarios  # noqa: E402

ORACLE = os.path.join(REPO, "oracle", "_build", "libgossip_oracle.so")


def digest(snapshot):
    out = {"counters": snapshot["counters"]}
    for k, v in snapshot.items():
        if k in ("counters", "node_range", "edge_range"):
            continue
        h = hashlib.sha256()
        if k == "deliv":
            for hop, frm in v:
                h.update(np.ascontiguousarray(hop).tobytes())
                h.update(np.ascontiguousarray(frm).tobytes())
        else:
            h.update(np.ascontiguousarray(scenarios._bits(v)).tobytes())
        out[k] = h.hexdigest()
    return out


def main():
    """Every scenario, or only the names given (merged into the file)."""
    path = os.path.join(HERE, "scenarios.json")
    names = sys.argv[1:]
    res = json.load(open(path)) if names and os.path.exists(path) else {}
    for name in names or sorted(scenarios.SCENARIOS):
        res[name] = digest(scenarios.run(ORACLE, name))
    with open(path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
