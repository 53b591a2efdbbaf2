#!/usr/bin/env python3
"""Per-kernel-instance PMC table from tools/archive/gpu_pmc_sq.sh output dirs.

    python tools/pmc_table.py gpurun_out/sq1 gpurun_out/sq2 ... [--filter conv]
"""
import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="conv")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for d in a.dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("ddmi::", "")
                    if a.filter not in name:
                        continue
                    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
                    cnt[name].add((d, r.get("Dispatch_Id")))
    for name, c in agg.items():
        print(f"== {name}")
        for k in sorted(c):
            print(f"   {k:28s} {c[k]:.4g}")
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA", "SQ_ACTIVE_INST_LDS"):
                if k in c:
                    print(f"   {k:28s} / WAVE_CYCLES = {c[k] / w:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_BUSY_CYCLES" in c:
            print(f"   MFMA_BUSY / BUSY_CYCLES = {c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_BUSY_CYCLES']:.3f}")
        if "TCC_HIT_sum" in c:
            print(f"   L2 hit rate = {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")


if __name__ == "__main__":
    main()
