#!/usr/bin/env python3
"""Determinism probe of the gathered value_proj: repeated forwards on the same inputs (eager first call, graph
replays after), value rows and trajectories compared call to call and against conv_x3 (DDMI_VALUE_SPLITK=0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402

B = int(os.environ.get("B", "3"))
sd = seeded_state_dict(None, 0) if False else None
from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
cfg = TransfuserConfig()
sd = seeded_state_dict(cfg, 0)
inp = synthetic_inputs(B, 17)
f = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"]).cuda()
names = [f"s{s}l{l}" for s in range(2) for l in range(2)]


def run(m):
    out = m.forward(f, noise=nz)["trajectory"].cpu().numpy()
    rows = {k: m.tap(f"value_taps_{k}").view(torch.int32).cpu().numpy()[: B * 640] for k in names}
    vals = {k: m.tap(f"value_rows_{k}").cpu().numpy()[: B * 640 * 256].reshape(-1, 256) for k in names}
    return out, rows, vals


res = []
for sp in os.environ.get("SPLITS", "1 2 3 3").split():
    os.environ["DDMI_VPROJ_SPLITS"] = sp
    m = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")
    res.append(run(m))
    m.close()
os.environ["DDMI_VALUE_SPLITK"] = "0"
m2 = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")
ref = run(m2)
m2.close()
for i, (out, rows, vals) in enumerate(res):
    line = [f"call {i}: traj vs call0 {np.abs(out - res[0][0]).max():.3e} vs x3 {np.abs(out - ref[0]).max():.3e}"]
    for k in names:
        live = rows[k] >= 0
        d0 = np.abs(vals[k][live] - res[0][2][k][live]).max()
        dx = np.abs(vals[k][live] - ref[2][k][live]).max()
        bad = np.where(np.abs(vals[k][live] - ref[2][k][live]).max(-1) > 1e-3)[0]
        line.append(f"{k}: live {int(live.sum())} d0 {d0:.2e} dx3 {dx:.2e} badrows {len(bad)} {bad[:6].tolist()}")
    print(" | ".join(line), flush=True)
