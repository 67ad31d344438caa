"""Per-kernel (or per-dispatch with --dispatch) averages of rocprofv3 PMC csv passes."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    per_dispatch = "--dispatch" in sys.argv
    for path in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        rows = list(csv.DictReader(open(path)))
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        ids = collections.defaultdict(set)
        dur = collections.defaultdict(float)
        for r in rows:
            k = r["Kernel_Name"].split("(")[0]
            if per_dispatch:
                k = k + "#" + r["Dispatch_Id"]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Dispatch_Id"] not in ids[k]:
                dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            ids[k].add(r["Dispatch_Id"])
        print("==", os.path.basename(os.path.dirname(path)))
        for k, d in agg.items():
            n = len(ids[k])
            print(f"{k} n={n} ms={dur[k]/n:.2f}", {c: f"{v / n:.4g}" for c, v in d.items()})


if __name__ == "__main__":
    main()
