"""Short fixed workload for PMC-counter passes: builds bench.py's engine,
runs `--warmup` rounds and then `--rounds` rounds (each rocprofv3 --pmc pass
runs this same program once)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config4", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--lib", default=None, help="another build of the product library (experiments)")
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    eng, _ = bench.build_engine(wl, a.warmup + a.rounds + 1, 3, 0, lib=a.lib)
    eng.step(1 + a.warmup * bench.HOPS_PER_ROUND)
    eng.sync()
    print("warm", eng.counters(), flush=True)
    eng.step(a.rounds * bench.HOPS_PER_ROUND)
    eng.sync()
    print("done", eng.counters(), flush=True)


if __name__ == "__main__":
    main()
