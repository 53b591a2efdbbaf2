#!/usr/bin/env python3
"""Per-kernel-class PMC summary of tools/gpu_pmc_round2.sh (profiles/<name>.md / .json).

    python tools/pmc_round2.py gpurun_out/pmc2 <name>

Counters are summed per kernel class over every dispatch of the run and divided by the dispatch count:
* MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): SQ_VALU_MFMA_BUSY_CYCLES
  counts matrix-pipe cycles summed over the SIMDs (32 per v_mfma_f32_32x32x16, MI355X_MICROARCH.md) and
  GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs, so GRBM / 8 is the kernel's clock count;
* LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all LDS-array cycles);
* HBM bytes = 2 x FETCH_SIZE (gfx950 reports half the bytes of 16-B/lane streaming reads) + WRITE_SIZE, in KB;
* L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kclass(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    n = re.sub(r"^void\s+", "", n).replace("ddmi::", "")
    # the gathered value_proj (conv_x3's GATHER = 1 instance: the decoder's cross-BEV attention contraction)
    # (round 5: the union-staged form; the gathered form behind it only computes the tiles whose union overflowed)
    if re.match(r"conv_x3_kernel<(\s*\d+\s*,){6}\s*1\s*>", n) or n.startswith("vproj_union_kernel"):
        return "value_proj"
    if n.startswith("vproj_kernel"):
        return "value_proj_fallback"
    return re.sub(r"<.*>", "", n).replace("_kernel", "")


def main():
    src, name = sys.argv[1], sys.argv[2]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for p in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = kclass(r["Kernel_Name"])
                c = r["Counter_Name"]
                agg[k][c] += float(r["Counter_Value"])
                disp[k][c].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    rows = {}
    for k, cs in agg.items():
        per = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
        d = {"dispatches": max(len(s) for s in disp[k].values()), "per_dispatch": per}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in per and per.get("GRBM_GUI_ACTIVE"):
            d["mfma_util"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / (per["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if per.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_share"] = per.get("SQ_LDS_BANK_CONFLICT", 0) / per["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in per or "WRITE_SIZE" in per:
            d["hbm_kb"] = 2 * per.get("FETCH_SIZE", 0) + per.get("WRITE_SIZE", 0)
        if per.get("TCC_HIT_sum", 0) + per.get("TCC_MISS_sum", 0):
            d["l2_hit"] = per["TCC_HIT_sum"] / (per["TCC_HIT_sum"] + per["TCC_MISS_sum"])
        rows[k] = d
    order = sorted(rows, key=lambda k: -rows[k]["per_dispatch"].get("GRBM_GUI_ACTIVE", 0) * rows[k]["dispatches"])
    lines = [f"# PMC per kernel class: {name}", "",
             "Bench workload (B = 64, f16x3, single-stream replays); values per dispatch, averaged over the run.",
             "", "| kernel | dispatches | MFMA util | MFMA busy cyc | GRBM_GUI_ACTIVE | LDS conflict share | "
             "HBM KB (2 FETCH + WRITE) | L2 hit |", "|---|---|---|---|---|---|---|---|"]
    f = lambda v, fmt: (fmt % v) if v is not None else "-"
    for k in order:
        d, per = rows[k], rows[k]["per_dispatch"]
        lines.append(f"| {k} | {d['dispatches']} | {f(d.get('mfma_util'), '%.3f')} | "
                     f"{f(per.get('SQ_VALU_MFMA_BUSY_CYCLES'), '%.3g')} | {f(per.get('GRBM_GUI_ACTIVE'), '%.3g')} | "
                     f"{f(d.get('lds_conflict_share'), '%.3f')} | {f(d.get('hbm_kb'), '%.0f')} | {f(d.get('l2_hit'), '%.3f')} |")
    out = os.path.join(ROOT, "profiles", name)
    open(out + ".md", "w").write("\n".join(lines) + "\n")
    json.dump(rows, open(out + ".json", "w"), indent=1)
    print("\n".join(lines[:20]))


if __name__ == "__main__":
    main()
