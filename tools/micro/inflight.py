"""Batches in flight: K forwards of B=64 on one handle (one stream) against the same K forwards
alternating over N handles, each on its own caller stream (N batches in flight: one batch's
low-occupancy phases - the per-scene decoder megakernels, the GPT stages - overlap the next
batch's trunk). Prints scenes/s per configuration and the waypoint agreement of the outputs.

    python tools/micro/inflight.py [--steps 100] [--n 2,3] [--single-stream]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--n", default="2,3")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--single-stream", action="store_true",
                    help="DDMI_STREAMS=0 for every handle (one handle queue each instead of two)")
    args = ap.parse_args()
    if args.single_stream:
        os.environ["DDMI_STREAMS"] = "0"
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    cfg = TransfuserConfig()
    sd = seeded_state_dict(cfg, 0)
    ns = [int(x) for x in args.n.split(",")]
    models = [DiffusionDriveModel(cfg, sd, device=0) for _ in range(max(ns))]
    inp = synthetic_inputs(args.batch, 1234, cfg)
    keys = ("camera_feature", "lidar_feature", "status_feature")
    feats = {k: torch.from_numpy(inp[k]).to(dev) for k in keys}
    noise = torch.from_numpy(inp["noise"]).to(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(max(ns))]

    def run(n, k):
        outs = [None] * n
        for i in range(k):
            j = i % n
            outs[j] = models[j].forward(feats, noise=noise, stream=streams[j])["trajectory"]
        return outs

    def timed(n, k):
        run(n, 2 * n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs = run(n, k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, outs

    ref = None
    for rep in range(2):
        for n in [1] + ns:
            dt, outs = timed(n, args.steps)
            o = outs[0].cpu().numpy()
            if ref is None:
                ref = o
            d = float(np.abs(o - ref).max())
            print(f"rep {rep} in_flight {n}: {args.batch * args.steps / dt:8.1f} scenes/s  "
                  f"{dt / args.steps * 1e3:6.3f} ms/step  max|d| vs 1: {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
