"""GPU debug: decoder megakernel vs the unfused chain, tap by tap (B = 2)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from diffusiondrive_amd.config import TransfuserConfig
from diffusiondrive_amd.model import DiffusionDriveModel
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs

cfg = TransfuserConfig()
sd = seeded_state_dict(cfg, 0)
B = 2
inp = synthetic_inputs(B, 31)
feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"])
res = {}
for mk in ("1", "0"):
    os.environ["DDMI_DECODER_MK"] = mk
    m = DiffusionDriveModel(cfg, sd, device=0, gemm="f16x3")
    out = m.forward(feats, noise=nz, steps=int(os.environ.get("STEPS", "2")))["trajectory"].numpy()
    torch.cuda.synchronize()
    d = {"traj": out}
    for name in ["traj_feature", "pts", "pts_next", "ddim_img"] + [f"{k}_s{s}l{l}" for k in ("gs", "reg", "cls", "value_slots") for s in range(2) for l in range(2)]:
        try:
            d[name] = m.tap(name).cpu().numpy()
        except Exception as e:
            d[name] = None
    res[mk] = d
    m.close()
n = {"traj_feature": B * 20 * 256, "pts": B * 160 * 2, "pts_next": B * 160 * 2, "ddim_img": B * 160 * 2, "traj": B * 24}
for k in res["1"]:
    a, b = res["1"][k], res["0"][k]
    if a is None or b is None:
        print(k, "missing", a is None, b is None)
        continue
    cnt = n.get(k, B * 20 * (24 if k.startswith("reg") else 256 if k.startswith("gs") else 640 if k.startswith("value") else 1))
    a, b = a[:cnt], b[:cnt]
    if k.startswith("value_slots"):
        a = a.view(np.int32); b = b.view(np.int32)
        print(f"{k:16s} equal {np.array_equal(a, b)}  mk[:8] {a[:8]} ref[:8] {b[:8]}")
        continue
    err = np.abs(a.astype(np.float64) - b).max()
    print(f"{k:16s} max abs err {err:.3e}  mk[:4] {a[:4]} ref[:4] {b[:4]}")

# CPU restatement of step 0's traj_feature from the step-0 points (run with STEPS=1)
if os.environ.get("STEPS") == "1":
    import torch.nn.functional as F
    pts = torch.from_numpy(res["1"]["pts"][: B * 160 * 2].reshape(B * 20, 8, 2))
    dim_t = torch.tensor([10000.0 ** (j / 16.0) for j in range(16)], dtype=torch.float32).repeat_interleave(2)
    def emb1(v):
        a = (v[..., None] * 6.283185307179586) / dim_t
        return torch.stack([a[..., 0::2].sin(), a[..., 1::2].cos()], -1).flatten(-2)
    emb = torch.cat([emb1(pts[..., 1]), emb1(pts[..., 0])], -1).reshape(B * 20, 512)
    g = lambda k: torch.from_numpy(np.asarray(sd["_trajectory_head." + k]))
    h = F.relu(emb @ g("plan_anchor_encoder.0.weight").T + g("plan_anchor_encoder.0.bias"))
    h = F.layer_norm(h, (256,), g("plan_anchor_encoder.2.weight"), g("plan_anchor_encoder.2.bias"))
    tfe = h @ g("plan_anchor_encoder.3.weight").T + g("plan_anchor_encoder.3.bias")
    for mk in ("1", "0"):
        t = res[mk]["traj_feature"][: B * 20 * 256].reshape(B * 20, 256)
        print("tfe cpu vs mk=" + mk, float(np.abs(t - tfe.numpy()).max()), t[0, :4], tfe[0, :4].numpy())
