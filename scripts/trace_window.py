"""Average kernel durations over the timed window of a rocprofv3 kernel trace:
the last `--hops` dispatches of each hop kernel (bench.py's timed region is
the last steps*10 hops of the run).  usage: trace_window.py run_kernel_trace.csv --hops 20"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--hops", type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"].split("(")[0]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print("kernel,dispatches_in_window,avg_ms")
    for k, v in sorted(by.items()):
        v.sort()
        per_hop = "k_phase_a<" in k or "k_phase_b<" in k or k in ("k_fwd", "void k_score_rows<1>",
                                                                   "void k_score_rows<2>")
        w = v[-a.hops:] if per_hop else v[-max(1, a.hops // 10):]
        print(f"{k},{len(w)},{sum(e - s for s, e in w) / len(w) / 1e6:.4f}")


if __name__ == "__main__":
    main()
