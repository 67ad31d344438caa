"""Summarise a rocprofv3 run: per-kernel calls / total / average / min / max
duration (ms) and register + LDS footprint, from either the rocpd SQLite
database (default output of rocprofv3 on ROCm 7.x) or a kernel_stats.csv.

usage: python scripts/prof_summary.py <run_results.db | *_kernel_stats.csv> [out.csv]
"""
import csv
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, vgpr_count, sgpr_count, lds_size from kernels").fetchall()
    agg = {}
    for name, dur, vgpr, sgpr, lds in rows:
        a = agg.setdefault(name, dict(name=name, calls=0, total_ms=0.0, min_ms=1e30, max_ms=0.0,
                                      vgpr=vgpr, sgpr=sgpr, lds=lds))
        ms = dur / 1e6
        a["calls"] += 1
        a["total_ms"] += ms
        a["min_ms"] = min(a["min_ms"], ms)
        a["max_ms"] = max(a["max_ms"], ms)
    out = sorted(agg.values(), key=lambda a: -a["total_ms"])
    for a in out:
        a["avg_ms"] = a["total_ms"] / a["calls"]
    return out


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append(dict(name=r["Name"], calls=int(r["Calls"]), total_ms=float(r["TotalDurationNs"]) / 1e6,
                            avg_ms=float(r["AverageNs"]) / 1e6, min_ms=float(r["MinNs"]) / 1e6,
                            max_ms=float(r["MaxNs"]) / 1e6, vgpr="", sgpr="", lds=""))
    return out


def main():
    src = sys.argv[1]
    rows = from_db(src) if src.endswith(".db") else from_csv(src)
    total = sum(r["total_ms"] for r in rows)
    fields = ["name", "calls", "total_ms", "avg_ms", "min_ms", "max_ms", "pct", "vgpr", "sgpr", "lds"]
    dst = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(dst, fieldnames=fields)
    w.writeheader()
    for r in rows:
        r["pct"] = round(100.0 * r["total_ms"] / total, 2)
        for k in ("total_ms", "avg_ms", "min_ms", "max_ms"):
            r[k] = round(r[k], 4)
        w.writerow({k: r[k] for k in fields})
    if dst is not sys.stdout:
        dst.close()
        print("wrote", os.path.abspath(sys.argv[2]))


if __name__ == "__main__":
    main()
