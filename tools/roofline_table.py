#!/usr/bin/env python3
"""Per-kernel-class roofline evidence: HBM GB/s and MFMA busy of every class of the bench forward.

    python tools/roofline_table.py profiles/<pmc>.json profiles/<trace>.json profiles/<out>.md

Joins a PMC summary (tools/pmc_round2.py: HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE and MFMA busy per dispatch, from
separate --pmc passes) with a kernel-trace summary of the same build (average duration per dispatch from
rocprofv3 --kernel-trace). achieved GB/s = HBM bytes per dispatch / average duration; the HBM peak is
MI355X_MICROARCH.md's 8 TB/s. MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).
"""
import json
import sys

HBM_PEAK = 8000.0  # GB/s
# trace class -> PMC class (the two summaries name the gathered value_proj and a few classes differently)
ALIAS = {"vproj_union": "value_proj", "value_proj": "value_proj_fallback"}  # round 5 class names


def main():
    pmc_path, trace_path, out = sys.argv[1:4]
    pmc = json.load(open(pmc_path))
    tr = json.load(open(trace_path))
    per_fwd = tr["dispatches"] and tr["per_forward_device_ms"] / tr["total_device_ms"]
    rows = []
    for cls, t in tr["classes"].items():
        p = pmc.get(ALIAS.get(cls, cls))
        if p is None or t["avg_us"] <= 0:
            continue
        mb = p.get("hbm_kb", 0.0) * 1024 / 1e6
        gbs = mb / 1e3 / (t["avg_us"] * 1e-6)
        rows.append((t["total_ms"] * per_fwd, cls, t["launches"] * per_fwd, t["avg_us"], mb, gbs,
                     p.get("mfma_util", 0.0), p.get("l2_hit", float("nan"))))
    rows.sort(reverse=True)
    lines = [f"# Roofline evidence per kernel class ({pmc_path.split('/')[-1]} + {trace_path.split('/')[-1]})", "",
             "HBM bytes from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (FETCH x 2), durations from the "
             "kernel trace of the same build; HBM peak 8 TB/s, MFMA busy against all 1024 SIMDs.", "",
             "| class | ms / forward | launches / forward | avg us | HBM MB / launch | HBM GB/s | of 8 TB/s | MFMA busy | L2 hit |",
             "|---|---|---|---|---|---|---|---|---|"]
    for ms, cls, n, us, mb, gbs, mf, l2 in rows:
        lines.append(f"| {cls} | {ms:.3f} | {n:.1f} | {us:.1f} | {mb:.1f} | {gbs:.0f} | {gbs / HBM_PEAK:.2f} | {mf:.2f} | "
                     f"{l2:.2f} |")
    txt = "\n".join(lines) + "\n"
    with open(out, "w") as f:
        f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
