#!/usr/bin/env python3
"""Per-kernel-class mean counter values per dispatch from rocprofv3 --pmc output directories.

    python tools/pmc_dump.py <dir> [<dir> ...] [--kernel substr]
"""
import argparse
import collections
import csv
import glob
import os
import re


def kclass(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    n = re.sub(r"^void\s+", "", n).replace("ddmi::", "")
    return re.sub(r"<.*>", "", n).replace("_kernel", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(p)):
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[key[0]] = r["Kernel_Name"]
            for (disp, ctr), v in per.items():
                vals[kclass(names[disp])][ctr].append(v)
    for k, ctrs in sorted(vals.items()):
        if a.kernel and a.kernel not in k:
            continue
        print(f"== {k}")
        for c, v in sorted(ctrs.items()):
            print(f"  {c:28s} {sum(v) / len(v):14.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
