#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel_stats.csv (every match under the given dirs): calls, average us, name (templated
names shortened). Usage: tools/kstats.py <dir> [<dir> ...] [--grep PATTERN]"""
import csv
import glob
import sys

args = sys.argv[1:]
pat = None
if "--grep" in args:
    i = args.index("--grep")
    pat = args[i + 1]
    args = args[:i] + args[i + 2:]
for d in args:
    for f in sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)):
        print(f"# {f}")
        for r in csv.DictReader(open(f)):
            n = r["Name"]
            if pat and pat not in n:
                continue
            short = n.replace("void ", "").replace("ddmi::", "").replace("(anonymous namespace)::", "").split("(")[0]
            print(f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.1f} us  {short}")
