"""Handle churn through the library alone (no pytest, no runner): create a two-stream handle, run it eager once, then
captured (instantiate + first launch) and replayed, destroy it; repeat. One line per iteration (flushed), so a
segfault's iteration is in the log. Diagnostic for DESIGN.md section 4 "Handle lifetime".

    python tools/repro/handle_churn.py <iterations> [heads 0|1] [batch] [long 0|1]
(run with DDMI_STREAM_POOL=0 to create / destroy the handles' streams per handle). long 1: the shape of the faulting
test order - a long-lived two-stream handle (B = 4) replayed every iteration while the others come and go, and after
the loop single-stream clones driven on torch streams (the runner / in-flight lanes), then the long-lived handle
destroyed and a fresh two-stream handle with heads run eager, captured and replayed.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402


def feats_of(B, cfg):
    inp = synthetic_inputs(B, 3, cfg)
    f = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    return f, torch.zeros(B, cfg.num_modes, cfg.trajectory_sampling.num_poses, 2).cuda()


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    heads = len(sys.argv) > 2 and sys.argv[2] == "1"
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    long_lived = len(sys.argv) > 4 and sys.argv[4] == "1"
    cfg = TransfuserConfig()
    sd = seeded_state_dict(cfg, 0)
    feats, noise = feats_of(B, cfg)
    ref = None
    base = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")  # never run: the weights blob for the clones
    keep = None
    if long_lived:
        keep = base.clone()
        f4, n4 = feats_of(4, cfg)
    for i in range(iters):
        m = base.clone()
        for _ in range(3):  # eager, captured (instantiate + first launch), replayed
            out = m.forward(feats, noise=noise, heads=heads)
        if keep is not None:
            keep.forward(f4, noise=n4)
        torch.cuda.synchronize()
        t = out["trajectory"].cpu()
        ref = t if ref is None else ref
        assert torch.equal(t, ref), i
        m.close()
        del m
        print(f"iter {i} ok (graph instantiations so far: {i + 1})", flush=True)
    if keep is not None:
        lanes = [base.clone() for _ in range(3)]
        streams = [torch.cuda.Stream() for _ in lanes]
        for m, s in zip(lanes, streams):
            m.set_streams(1)
            for _ in range(3):
                with torch.cuda.stream(s):
                    m.forward(feats, noise=noise, stream=s)
        torch.cuda.synchronize()
        for m in lanes:
            m.close()
        print("single-stream lanes on torch streams: ok", flush=True)
        keep.close()
        fresh = base.clone()
        for r in range(3):
            fresh.forward(feats, noise=noise, heads=True)
            torch.cuda.synchronize()
            print(f"fresh two-stream handle after the long-lived one: forward {r} ok", flush=True)
        fresh.close()
    print(f"handle_churn: {iters} handles, heads {int(heads)}, B {B}, long {int(long_lived)}: no fault", flush=True)


if __name__ == "__main__":
    main()
