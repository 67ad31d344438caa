"""Generates tests/golden/midsize.json: mid-size goldens of the benchmarked
configurations, made by the CPU oracle offline (minutes, too slow for the CPU
test suite) and compared bit-exactly with the GPU engine by
tests/test_midsize_gpu.py.

  c4mid   config4's workload (bench.build_engine: random 32-regular graph,
          64 topics, every peer in every topic, Eth2 scoring, 1000 msgs per
          round round-robin over the topics) at 30,000 peers: Join + 2 rounds
          of publishes + 1 round to drain.  E x T = 61M (edge, topic) pairs,
          W = 256 message words, 2048 pairs per node: the production kernel
          instantiations at 3% of the headline node count.
  c3mid   config3's workload (1 topic x 10048 slots) at 30,000 peers over 8
          rounds, into the MaxIHaveLength cut mode.

Each digest covers the counters, mesh, fanout, backoff, every score-counter
array, behaviour penalties, scores (float64 on their bit patterns) and the
per-node first-delivery hop and first deliverer of every 10th message.
Usage: python tests/golden/make_golden_mid.py [name ...]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REPO = os.path.dirname(TESTS)
for p in (os.path.join(REPO, "go-libp2p-pubsub_amd"), TESTS, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import bench  # noqa: E402
import scenarios  # noqa: E402
from make_golden import digest  # noqa: E402

ORACLE = os.path.join(REPO, "oracle", "_build", "libgossip_oracle.so")
PATH = os.path.join(HERE, "midsize.json")

MID = {
    "c4mid": dict(workload="config4", n=30_000, rounds=2, drain=1),
    "c3mid": dict(workload="config3", n=30_000, rounds=8, drain=1),
}


def run(lib, name):
    from pubsub_amd import WithRecordDeliveries
    m = MID[name]
    wl = dict(bench.WORKLOADS[m["workload"]], n=m["n"])
    e, _ = bench.build_engine(wl, m["rounds"], 3, 0, lib=lib, extra=(WithRecordDeliveries(),))
    e.step(1 + (m["rounds"] + m["drain"]) * bench.HOPS_PER_ROUND)
    return scenarios.snapshot(e, range(0, e.n_published, 10))


def main():
    names = sys.argv[1:] or sorted(MID)
    res = json.load(open(PATH)) if os.path.exists(PATH) else {}
    for name in names:
        t0 = time.time()
        res[name] = digest(run(ORACLE, name))
        print(name, f"{time.time() - t0:.0f} s", res[name]["counters"], flush=True)
        with open(PATH, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", PATH)


if __name__ == "__main__":
    main()
