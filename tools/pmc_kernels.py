#!/usr/bin/env python3
"""Per-kernel-instantiation PMC summary (tools/pmc_round2.py's formulas, keyed by the full template name instead of the
kernel class): python tools/pmc_kernels.py <dir> [--grep PATTERN]. Prints dispatches, MFMA utilisation, LDS conflict
share, HBM MB per dispatch (2 x FETCH_SIZE + WRITE_SIZE) and L2 hit rate for the counters present."""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
pat = sys.argv[sys.argv.index("--grep") + 1] if "--grep" in sys.argv else None
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for p in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].replace("void ", "").replace("ddmi::", "").replace("(anonymous namespace)::", "").split("(")[0]
        if pat and pat not in n:
            continue
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n][r["Counter_Name"]].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
for n, cs in sorted(agg.items()):
    per = {c: v / max(1, len(disp[n][c])) for c, v in cs.items()}
    out = [f"{n:40s} disp {max(len(s) for s in disp[n].values()):4d}"]
    if per.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in per:
        out.append(f"mfma {per['SQ_VALU_MFMA_BUSY_CYCLES'] / (per['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    if per.get("SQ_LDS_IDX_ACTIVE"):
        out.append(f"lds_conf {per.get('SQ_LDS_BANK_CONFLICT', 0) / per['SQ_LDS_IDX_ACTIVE']:.3f}")
    if "FETCH_SIZE" in per:
        out.append(f"read_MB {2 * per['FETCH_SIZE'] / 1e3:.1f}")
    if "WRITE_SIZE" in per:
        out.append(f"write_MB {per['WRITE_SIZE'] / 1e3:.1f}")
    if per.get("TCC_HIT_sum", 0) + per.get("TCC_MISS_sum", 0):
        out.append(f"l2_hit {per['TCC_HIT_sum'] / (per['TCC_HIT_sum'] + per['TCC_MISS_sum']):.3f}")
    print("  ".join(out))
