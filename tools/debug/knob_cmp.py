"""GPU diagnostics: B = 64 f16x3 forward with an env knob on / off: agent_states, trajectory and a few taps
against the committed B = 64 golden.   python tools/debug/knob_cmp.py DDMI_GPT_ATTN_X3"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from diffusiondrive_amd.config import TransfuserConfig
from diffusiondrive_amd.model import DiffusionDriveModel
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
knob = sys.argv[1]
cfg = TransfuserConfig()
sd = seeded_state_dict(cfg, 0)
B = 64
inp = synthetic_inputs(B, 1234)
feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"])
g = np.load(os.path.join(ROOT, "tests", "golden", "ref_b64_s1234.npz"))
outs = {}
for v in ("1", "0"):
    os.environ[knob] = v
    m = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")
    out = m.forward(feats, noise=nz, heads=True)
    outs[v] = {k: out[k].numpy() for k in ("agent_states", "trajectory")}
    outs[v]["query_out"] = m.tap("query_out").cpu().numpy()[: B * 31 * 256]
    outs[v]["bev_feature"] = m.tap("bev_feature").cpu().numpy()
    del m
for v in ("1", "0"):
    d = np.abs(outs[v]["agent_states"] - g["agent_states"])
    i = np.unravel_index(d.argmax(), d.shape)
    print(f"{knob}={v}: agent_states max err {d.max():.3e} at {i}; trajectory max err "
          f"{np.abs(outs[v]['trajectory'] - g['trajectory']).max():.3e}")
for k in ("query_out", "bev_feature"):
    a, b = outs["1"][k], outs["0"][k]
    n = min(a.size, b.size)
    print(f"{k}: on-vs-off max abs {np.abs(a[:n] - b[:n]).max():.3e} max|x| {np.abs(b[:n]).max():.3e}")
