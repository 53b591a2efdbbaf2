#!/usr/bin/env python3
"""Write the HBM-traffic record bench.py reads (profiles/pmc_<kernel>_<gemm>.json) from a PMC summary.

    python tools/pmc_traffic.py profiles/<pmc_summary>.json <round tag> [--bench profiles/<bench>.json]

<pmc_summary>.json is tools/pmc_round2.py's output over tools/gpu_pmc_round2.sh's passes (separate rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE runs over the bench workload, single-stream replays). HBM bytes per dispatch =
2 x FETCH_SIZE + WRITE_SIZE (KB; gfx950 reports half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md).
With --bench (a bench.py JSON line of the same build) the algorithmic bytes per launch and the
traffic / algorithmic ratio are recorded beside it.
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("tag")
    ap.add_argument("--bench")
    ap.add_argument("--kernel", default="conv_x6")
    ap.add_argument("--gemm", default="f16x3")
    args = ap.parse_args()
    rows = json.load(open(args.summary))
    d = rows[args.kernel]
    per = d["per_dispatch"]
    rec = {
        "kernel": args.kernel,
        "gemm": args.gemm,
        "measured": args.tag,
        "source": f"{os.path.relpath(args.summary, ROOT)} (tools/gpu_pmc_round2.sh: separate rocprofv3 --pmc "
                  f"FETCH_SIZE / WRITE_SIZE passes over the bench workload, single-stream replays)",
        "dispatches": d["dispatches"],
        "hbm_bytes_per_launch": d["hbm_kb"] * 1024.0,
        "fetch_bytes_per_launch_x2": 2 * per.get("FETCH_SIZE", 0.0) * 1024.0,
        "write_bytes_per_launch": per.get("WRITE_SIZE", 0.0) * 1024.0,
        "mfma_util": d.get("mfma_util"),
        "lds_conflict_share": d.get("lds_conflict_share"),
        "l2_hit": d.get("l2_hit"),
    }
    if args.bench:
        b = json.loads(open(args.bench).read().strip().splitlines()[-1])
        alg = b["roofline"]["algorithmic_bytes_per_launch"]
        rec["algorithmic_bytes_per_launch"] = alg
        rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / alg
        rec["algorithmic_note"] = ("input map + output + residual + weight image of each launch counted once, "
                                   "averaged over the forward's launches (runtime.cpp conv_algo_bytes)")
    out = os.path.join(ROOT, "profiles", f"pmc_{args.kernel}_{args.gemm}.json")
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
