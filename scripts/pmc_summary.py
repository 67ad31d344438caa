"""Steady-state per-launch HBM traffic from rocprofv3 PMC passes (FETCH_SIZE /
WRITE_SIZE, KiB units) for each kernel: mean over the last `--last` dispatches.
Applies the gfx950 correction FETCH_SIZE x 2: MI355X_MICROARCH.md states it for
16-B-per-lane streaming reads, and scripts/pmc_calib.hip measured the same
exact 1/2 for 4- and 8-byte-per-lane reads and for a u32 read-modify-write
(profiles/r02_pmc_calib/), the widths the engine's kernels use; WRITE_SIZE
is exact at all three widths.  The raw value is kept too.
usage: pmc_summary.py gpurun_out/<tag> out.json"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(dict)
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0]
        d[k][int(r["Dispatch_Id"])] = (float(r["Counter_Value"]),
                                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return d


def main():
    root, out = sys.argv[1], sys.argv[2]
    last = 10
    f = per_dispatch(os.path.join(root, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_dispatch(os.path.join(root, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in f:
        fv = [f[k][i] for i in sorted(f[k])][-last:]
        wv = [w[k][i] for i in sorted(w.get(k, {}))][-last:]
        fk = sum(x[0] for x in fv) / len(fv)
        wk = sum(x[0] for x in wv) / len(wv) if wv else 0.0
        res[k] = {"dispatches": len(fv), "dispatches_total": len(f[k]), "last_dispatch": max(f[k]),
                  "fetch_kib_raw": round(fk), "write_kib": round(wk),
                  "read_bytes_est": int(2 * fk * 1024), "write_bytes": int(wk * 1024),
                  "traffic_bytes_est": int(2 * fk * 1024 + wk * 1024),
                  "ms_under_pmc": round(sum(x[1] for x in fv) / len(fv), 3)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
