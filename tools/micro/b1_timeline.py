#!/usr/bin/env python3
"""Per-forward timeline from a kernel trace of tools/micro/b1_trace.py: forwards split at host gaps > 1 ms; for
the median forward, every launch's start / end offset (us), duration, class and queue, plus per-class busy time.

    python tools/micro/b1_timeline.py <trace_dir> [--out file.md]"""
import argparse
import collections
import csv
import glob
import re


def kname(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    n = re.sub(r"^void\s+", "", n).replace("ddmi::", "")
    return re.sub(r"_kernel\b", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    f = glob.glob(f"{a.trace_dir}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    fw, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > 1_000_000:
            fw.append(cur)
            cur = []
        cur.append(r)
        last_end = e if last_end is None else max(last_end, e)
    fw.append(cur)
    walls = [(max(int(r["End_Timestamp"]) for r in x) - int(x[0]["Start_Timestamp"])) / 1e3 for x in fw]
    order = sorted(range(len(fw)), key=lambda i: walls[i])
    mid = order[len(order) // 2]
    x = fw[mid]
    t0 = int(x[0]["Start_Timestamp"])
    lines = [f"forwards {len(fw)}; device walls us: " + " ".join(f"{w:.0f}" for w in walls),
             f"median forward #{mid}: {walls[mid]:.1f} us, {len(x)} launches", "",
             "| start | end | dur | kernel | grid | queue |", "|---|---|---|---|---|---|"]
    busy = collections.defaultdict(float)
    for r in x:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        k = kname(r["Kernel_Name"])
        busy[re.sub(r"<.*", "", k)] += e - s
        g = r.get("Grid_Size_X", r.get("Grid_Size", ""))
        lines.append(f"| {s:.1f} | {e:.1f} | {e - s:.1f} | {k[:70]} | {g} | {r.get('Queue_Id', '')} |")
    lines += ["", "| class | busy us |", "|---|---|"]
    lines += [f"| {k} | {v:.1f} |" for k, v in sorted(busy.items(), key=lambda kv: -kv[1])]
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
