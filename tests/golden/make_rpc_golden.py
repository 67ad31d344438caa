"""Writes tests/golden/rpc_fragment.json: the shapes of the RPCs that the
reference's TestFragmentRPCFunction (gossipsub_test.go:2085-2250) fragments,
plus 10 seeded random RPCs, each with the oracle's fragmentRPC result
(oracle/oracle_rpc.py) at several limits.  Run from the repo root:
    python tests/golden/make_rpc_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "go-libp2p-pubsub_amd")]
import oracle_rpc as O  # noqa: E402
import test_rpc_fragment as T  # noqa: E402


def shape_dict(rpc):
    s = T.shape_of(rpc)
    return {k: getattr(s, k) for k in ("sub_size", "pub_size", "has_control", "ihave_topic_len",
                                        "ihave_ids", "iwant_ids", "graft_size", "prune_size")}


def result(rpc, limit):
    try:
        frags = O.fragment_rpc(rpc, limit)
    except ValueError as e:
        return {"error": str(e)}
    return {"frag_size": [O.size(r) for r in frags]}


def main():
    cases = []
    for name, rpc in T.reference_case_rpcs():
        cases.append({"name": name, "shape": shape_dict(rpc), "limit": T.LIMIT,
                      **result(rpc, T.LIMIT)})
    for seed in range(10):
        rpc = T.random_rpc(random.Random(1000 + seed))
        for limit in (300, 1024, 4096):
            cases.append({"name": f"random{seed}_{limit}", "shape": shape_dict(rpc), "limit": limit,
                          **result(rpc, limit)})
    with open(os.path.join(HERE, "rpc_fragment.json"), "w") as f:
        json.dump(cases, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
