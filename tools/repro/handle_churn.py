"""Handle churn through the library alone (no pytest, no runner): create a two-stream handle, run it eager once, then
captured (instantiate + first launch) and replayed, destroy it; repeat. One line per iteration (flushed), so a
segfault's iteration is in the log. Diagnostic for DESIGN.md section 4 "Handle lifetime".

    python tools/repro/handle_churn.py <iterations> [heads 0|1] [batch]
(run with DDMI_STREAM_POOL=0 to create / destroy the handles' streams per handle)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    heads = len(sys.argv) > 2 and sys.argv[2] == "1"
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    cfg = TransfuserConfig()
    sd = seeded_state_dict(cfg, 0)
    inp = synthetic_inputs(B, 3, cfg)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    noise = torch.zeros(B, cfg.num_modes, cfg.trajectory_sampling.num_poses, 2).cuda()
    ref = None
    base = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")  # never run: the weights blob for the clones
    for i in range(iters):
        m = base.clone()
        for _ in range(3):  # eager, captured (instantiate + first launch), replayed
            out = m.forward(feats, noise=noise, heads=heads)
        torch.cuda.synchronize()
        t = out["trajectory"].cpu()
        ref = t if ref is None else ref
        assert torch.equal(t, ref), i
        m.close()
        del m
        print(f"iter {i} ok (graph instantiations so far: {i + 1})", flush=True)
    print(f"handle_churn: {iters} handles, heads {int(heads)}, B {B}: no fault", flush=True)


if __name__ == "__main__":
    main()
