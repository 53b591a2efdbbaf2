"""GPU diagnostics: tf-decoder megakernel vs the unfused chain at B = 64 (f16x3), per tensor, plus agent_states
against the committed B = 64 golden."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from diffusiondrive_amd.config import TransfuserConfig
from diffusiondrive_amd.model import DiffusionDriveModel
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
cfg = TransfuserConfig()
sd = seeded_state_dict(cfg, 0)
B = 64
inp = synthetic_inputs(B, 1234)
feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"])
g = np.load(os.path.join(ROOT, "tests", "golden", "ref_b64_s1234.npz"))
sizes = {"query_out": B * 31 * 256, "agent_kv0": B * 30 * 512, "ego_out0": B * 256, "ego_out1": B * 256}
res = {}
for mk in ("1", "0"):
    os.environ["DDMI_TFDEC_MK"] = mk
    m = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")
    out = m.forward(feats, noise=nz, heads=True)
    res[mk] = ({k: m.tap(k).cpu().numpy()[:n] for k, n in sizes.items()}, out["agent_states"].numpy())
    del m
for k in sizes:
    a, b = res["1"][0][k], res["0"][0][k]
    print(f"{k:10s} mk-vs-unfused max abs {np.abs(a - b).max():.3e}  max|x| {np.abs(b).max():.3e}")
for mk in ("1", "0"):
    d = np.abs(res[mk][1] - g["agent_states"])
    i = np.unravel_index(d.argmax(), d.shape)
    print(f"agent_states vs golden (mk={mk}): max {d.max():.3e} at {i}, value {g['agent_states'][i]:.4f}")
