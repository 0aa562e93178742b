"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(paths):
    agg = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for p in paths:
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(p)):
            k = r.get("Kernel_Name", "")
            d = r.get("Dispatch_Id", "")
            per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, d), cs in per.items():
            for c, v in cs.items():
                agg[k][c].append(v)
    return agg


def short(k):
    for tag in ("k_tracescreen", "k_camerarays", "k_cell_depths", "k_shard_copy", "k_march", "k_shade", "k_finish", "k_primary"):
        if tag in k:
            return tag + ("<stats>" if "true" in k else "")
    return k[:40]


if __name__ == "__main__":
    d = sys.argv[1]
    agg = load(glob.glob(os.path.join(d, "*", "run_counter_collection.csv")))
    for k, cs in sorted(agg.items()):
        print(short(k))
        for c, vs in sorted(cs.items()):
            print(f"   {c:28s} {sum(vs) / len(vs):.4g}  (n={len(vs)})")
