#!/usr/bin/env python3
"""The one-channel LiDAR stem (DDMI_STEM1=1) against the 4-channel form on the bench's B = 64 golden batch (GPU):
the pooled LiDAR stem map, the LiDAR trunk taps, and every per-(step, layer) reg / cls against the reference golden,
with the (scene, mode) where each reg error peaks. Each form on a fresh handle (the knob is read per dispatch)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_util import load  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402
from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402

g = load(os.path.join(ROOT, "tests", "golden", "ref_b64_s1234.npz"))
B = 64
inp = synthetic_inputs(B, 1234)
feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
sd = seeded_state_dict(TransfuserConfig(), 0)
res = {}
for form in ("0", "1"):
    os.environ["DDMI_STEM1"] = form
    m = DiffusionDriveModel(state_dict=sd, device=0, gemm="f16x3")
    out = m.forward(feats, noise=torch.from_numpy(inp["noise"]), modes=True)
    r = {"pool": m.tap("lid_pool").cpu().numpy().copy(), "traj": out["trajectory"].numpy()}
    for s in range(2):
        for l in range(2):
            r[f"reg_s{s}l{l}"] = m.tap(f"reg_s{s}l{l}", (B, 20, 8, 3)).cpu().numpy().copy()
            r[f"cls_s{s}l{l}"] = m.tap(f"cls_s{s}l{l}", (B, 20)).cpu().numpy().copy()
    r["flags"] = m.numerics_flags()
    m.close()
    res[form] = r
for form, r in res.items():
    line = [f"DDMI_STEM1={form} flags {r['flags']}"]
    if form != "0":
        d = np.abs(r["pool"] - res["0"]["pool"])
        line.append(f"pool vs 4ch max {d.max():.3e} (rel {d.max() / np.abs(res['0']['pool']).max():.2e}), "
                    f"nonzero {np.count_nonzero(d)} of {d.size}")
    for k in [f"reg_s{s}l{l}" for s in range(2) for l in range(2)]:
        e = np.abs(r[k] - g[k])
        idx = np.unravel_index(int(e.argmax()), e.shape)
        dd = np.abs(r[k] - res["0"][k]).max()
        line.append(f"{k}: vs golden {e.max():.3e} at scene {idx[0]} mode {idx[1]} pose {idx[2]} comp {idx[3]}; "
                    f"vs 4ch {dd:.3e}")
    print("\n  ".join(line), flush=True)
