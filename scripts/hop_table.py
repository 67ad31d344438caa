"""Per-dispatch durations (ms) of the last hops' kernels from a rocprofv3
kernel trace (csv or rocpd .db).  usage: hop_table.py <trace.csv|results.db> [n]"""
import collections
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    out = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))]
    return sorted(out, key=lambda x: x[1])


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 22
    by = collections.defaultdict(list)
    for name, s, e in rows(path):
        by[name.split("(")[0]].append((e - s) / 1e6)
    for k, v in sorted(by.items()):
        print(f"{k} n={len(v)} last={[round(x, 2) for x in v[-n:]]}")


if __name__ == "__main__":
    main()
