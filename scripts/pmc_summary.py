#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per kernel (short names) over every pass directory given."""
import csv
import glob
import sys
from collections import defaultdict


def short(n):
    if "gemm_w4" in n:
        return "w4"
    if "gemm256" in n:
        return "gemm256"
    if n.startswith("Custom_Cijk") or n.startswith("Cijk"):
        return "hipblaslt:" + ("MT" + n.split("_MT")[1].split("_")[0] if "_MT" in n else n[:30])
    return n[:40]


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", ""))
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(f"== {k}")
        for c, vs in sorted(cs.items()):
            print(f"   {c:28s} {sum(vs) / len(vs):16.4g}  (n={len(vs)})")


if __name__ == "__main__":
    main()
