#!/usr/bin/env python3
"""Summarise rocprofv3 output (kernel trace/stats CSV or rocpd SQLite) into profiles/.

    python tools/prof_summary.py <rocprof_out_dir> <name> [--forwards N] [--pmc <pmc_dir> ...]

Writes profiles/<name>.md (human summary) and profiles/<name>.json. Kernel template instances
are grouped into classes (conv_gemm<2,2,0> ... -> conv_gemm) so the per-class average launch
duration can be compared with bench.py's HIP-event roofline numbers. With --pmc dirs from
separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes, HBM bytes per conv_gemm launch
are derived per MI355X_MICROARCH.md (FETCH_SIZE x2 for 16-B/lane streaming reads on gfx950).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sqlite3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kclass(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    n = re.sub(r"^void\s+", "", n)
    n = n.replace("ddmi::", "")
    # the gathered value_proj (value_proj.hip, or conv_x3's GATHER = 1 instance): its own class, as in
    # tools/pmc_round2.py, so the trace and PMC summaries join per class (tools/roofline_table.py)
    if re.match(r"conv_x3_kernel<(\s*\d+\s*,){6}\s*1\s*>", n) or n.startswith("vproj_kernel"):
        return "value_proj"
    n = re.sub(r"<.*>", "", n)
    return n.replace("_kernel", "")


def load_trace(d):
    """[(name, start_ns, end_ns, grid_x, grid_z)] in start order."""
    rows = []
    csvs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if csvs:
        for p in csvs:
            with open(p) as f:
                for r in csv.DictReader(f):
                    rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                 int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), int(r.get("Grid_Size_Z", 1) or 1)))
    else:
        for p in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            c = sqlite3.connect(p)
            rows += c.execute("select name, start, end, grid_x, grid_z from kernels").fetchall()
    rows.sort(key=lambda r: r[1])
    return rows


def load_pmc(dirs):
    """{class: {counter: (sum, n)}} over all dispatches."""
    out = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    c = out[kclass(r["Kernel_Name"])][r["Counter_Name"]]
                    c[0] += float(r["Counter_Value"])
                    c[1] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("name")
    ap.add_argument("--forwards", type=int, default=0,
                    help="forward passes in the trace; by default derived from the trace itself (stem_pool launches / 2: "
                         "every forward runs the camera and the LiDAR stem once), and a given value that disagrees "
                         "with the trace is replaced by the trace's count")
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--note", default="")
    ap.add_argument("--pmc-kernel", default="conv_gemm", help="kernel class whose HBM bytes per launch to derive")
    a = ap.parse_args()
    rows = load_trace(a.trace_dir)
    if not rows:
        raise SystemExit(f"no kernel trace found under {a.trace_dir}")
    cls = collections.defaultdict(lambda: [0, 0.0])
    inst = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e, gx, gz in rows:
        cls[kclass(name)][0] += 1
        cls[kclass(name)][1] += (e - s) / 1e3
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "").replace("ddmi::", "")
        inst[short][0] += 1
        inst[short][1] += (e - s) / 1e3
    total_us = sum(v[1] for v in cls.values())
    res = {"note": a.note, "dispatches": len(rows), "total_device_ms": total_us / 1e3, "classes": {}, "instances": {}}
    for k, (n, us) in sorted(cls.items(), key=lambda x: -x[1][1]):
        res["classes"][k] = {"launches": n, "total_ms": us / 1e3, "avg_us": us / n, "share": us / total_us}
    for k, (n, us) in sorted(inst.items(), key=lambda x: -x[1][1]):
        res["instances"][k] = {"launches": n, "total_ms": us / 1e3, "avg_us": us / n}
    stems = cls.get("stem_pool", [0, 0.0])[0]
    derived = stems // 2 if stems and stems % 2 == 0 else 0
    if derived and a.forwards and a.forwards != derived:
        print(f"[prof_summary] --forwards {a.forwards} disagrees with the trace ({stems} stem_pool launches = "
              f"{derived} forwards): using {derived}")
    a.forwards = derived or a.forwards
    res["forwards"] = a.forwards
    res["forwards_source"] = "stem_pool launches / 2" if derived else ("--forwards" if a.forwards else None)
    if a.forwards:
        res["per_forward_device_ms"] = total_us / 1e3 / a.forwards
        for v in res["classes"].values():
            v["launches_per_forward"] = v["launches"] / a.forwards
            v["ms_per_forward"] = v["total_ms"] / a.forwards
    if a.pmc:
        pmc = load_pmc(a.pmc)
        res["pmc"] = {}
        for k, ctrs in pmc.items():
            res["pmc"][k] = {c: {"sum": v[0], "dispatches": v[1], "per_launch": v[0] / max(v[1], 1)}
                             for c, v in ctrs.items()}
        cg = res["pmc"].get(a.pmc_kernel, {})
        res["pmc_kernel"] = a.pmc_kernel
        if "FETCH_SIZE" in cg and "WRITE_SIZE" in cg:
            # FETCH_SIZE / WRITE_SIZE are in KB; gfx950 FETCH_SIZE counts half of wide streaming reads
            fetch = cg["FETCH_SIZE"]["per_launch"] * 1024 * 2
            write = cg["WRITE_SIZE"]["per_launch"] * 1024
            res["hbm_bytes_per_launch"] = fetch + write
            res["fetch_bytes_per_launch_x2"] = fetch
            res["write_bytes_per_launch"] = write
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", a.name + ".json"), "w") as f:
        json.dump(res, f, indent=1)
    lines = [f"# rocprofv3 summary: {a.name}", "", a.note, "",
             f"dispatches: {len(rows)}; total device time: {total_us / 1e3:.2f} ms"
             + (f"; forwards in the trace: {a.forwards} ({res['forwards_source']}); per forward: "
                f"{res['per_forward_device_ms']:.2f} ms" if a.forwards else ""), "",
             "| kernel class | launches | total ms | avg us | share | launches / forward | ms / forward |",
             "|---|---|---|---|---|---|---|"]
    for k, v in res["classes"].items():
        pf = (f"{v['launches_per_forward']:.1f} | {v['ms_per_forward']:.3f}" if a.forwards else "- | -")
        lines.append(f"| {k} | {v['launches']} | {v['total_ms']:.2f} | {v['avg_us']:.1f} | {100 * v['share']:.1f}% | {pf} |")
    lines += ["", "| kernel instance | launches | total ms | avg us |", "|---|---|---|---|"]
    for k, v in list(res["instances"].items())[:25]:
        lines.append(f"| `{k}` | {v['launches']} | {v['total_ms']:.2f} | {v['avg_us']:.1f} |")
    if a.pmc:
        lines += ["", "PMC (separate passes):", "", "| kernel class | counter | per launch |", "|---|---|---|"]
        for k, ctrs in res["pmc"].items():
            for c, v in ctrs.items():
                lines.append(f"| {k} | {c} | {v['per_launch']:.4g} |")
    with open(os.path.join(ROOT, "profiles", a.name + ".md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:20]))


if __name__ == "__main__":
    main()
