#!/usr/bin/env python3
"""Critical-path view of graph-replayed forwards from a rocprofv3 kernel trace.

    python tools/timeline.py <trace_dir> [--first-kernel stem_pool] [--nfwd 5]

Splits the trace into forwards at each launch of the first kernel of the forward, and for the
middle forwards reports: wall (first start -> last end), busy (union of kernel intervals), idle gaps,
and per-class device time with its share of the union (overlap makes the class sum exceed busy).
"""
import argparse
import collections
import csv
import glob
import os
import re


def kclass(name):
    name = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void\s+", "", name.split("(")[0]).replace("ddmi::", "")
    return re.sub(r"<.*>", "", n).replace("_kernel", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--first-kernel", default="nchw_to_nhwc")
    ap.add_argument("--skip", type=int, default=3, help="forwards before the graph replays (warmup/capture)")
    ap.add_argument("--count", type=int, default=5, help="graph-replayed forwards to analyse")
    a = ap.parse_args()
    p = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(((kclass(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                   for r in csv.DictReader(open(p))), key=lambda x: x[1])
    starts = [i for i, r in enumerate(rows) if r[0] == a.first_kernel]
    # nchw_to_nhwc runs twice per forward (camera, LiDAR): take every other
    starts = starts[::2]
    fw = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    fw = fw[a.skip:a.skip + a.count]  # the timed graph replays
    tot = collections.defaultdict(float)
    walls, busys = [], []
    for f in fw:
        t0, t1 = f[0][1], max(r[2] for r in f)
        walls.append((t1 - t0) / 1e6)
        iv = sorted((s, e) for _, s, e in f)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        busys.append(busy / 1e6)
        for k, s, e in f:
            tot[k] += (e - s) / 1e6 / len(fw)
    n = len(fw)
    print(f"forwards analysed: {n}; launches/forward {sum(len(f) for f in fw) / n:.0f}")
    print(f"wall {sum(walls) / n:.3f} ms, busy (union) {sum(busys) / n:.3f} ms, idle {sum(walls) / n - sum(busys) / n:.3f} ms")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {k:24s} {v:8.3f} ms")


if __name__ == "__main__":
    main()
