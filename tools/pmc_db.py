#!/usr/bin/env python3
"""Per-kernel PMC averages from rocprofv3 rocpd SQLite output (the default format when -f csv is not given).

    python tools/pmc_db.py <dir-with-*.db> [--kernel substring]
"""
import argparse
import collections
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: [0.0, 0])
    for d in a.dirs:
        for p in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            db = sqlite3.connect(p)
            q = ("select k.dispatch_id, k.kernel_name, e.counter_name, e.counter_value from pmc_events e "
                 "join counters_collection k on k.event_id = e.event_id")
            per = collections.defaultdict(float)  # (db, dispatch, counter) -> sum over instances
            for did, kn, cn, v in db.execute(q).fetchall():
                if a.kernel in (kn or ""):
                    per[(p, did, cn)] += float(v)
            for (_, _, cn), v in per.items():
                agg[cn][0] += v
                agg[cn][1] += 1
    print("counter                      per dispatch (summed over instances)")
    for k, (v, n) in sorted(agg.items()):
        print(f"{k:28s} {v / max(n, 1):14.6g}  (dispatches={n})")


if __name__ == "__main__":
    main()
