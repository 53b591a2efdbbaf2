#!/usr/bin/env python3
"""Per-launch timeline of one graph-replayed forward from a rocprofv3 kernel trace (start / end offsets in
us, duration, kernel class, queue), for reading which branch is on the critical path.

    python tools/tail_view.py <trace_dir> [--from-us T] [--fwd K]
"""
import argparse
import csv
import glob
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--from-us", type=float, default=0.0)
    ap.add_argument("--fwd", type=int, default=8, help="which forward (counted by its first nchw_to_nhwc pair)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(glob.glob(f"{a.trace_dir}/**/*kernel_trace.csv", recursive=True)[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r["Kernel_Name"]][::2]
    fw = rows[starts[a.fwd]:starts[a.fwd + 1]]
    t0 = int(fw[0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in fw)
    print(f"forward wall {(end - t0) / 1e3:.1f} us, {len(fw)} launches")
    for r in fw:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        if s >= a.from_us:
            n = re.sub(r"<.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0])
            n = n.replace("void ", "").replace("ddmi::", "")
            print(f"{s:9.1f} {e:9.1f} {e - s:7.1f} {n[:28]:28s} q={r['Queue_Id']} grid={r['Grid_Size_X']}")


if __name__ == "__main__":
    main()
