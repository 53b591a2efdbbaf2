"""GPU diagnostics: per-phase shader-clock stamps of the tf-decoder megakernel (DDMI_MK_STAMPS=1), B = 64."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["DDMI_MK_STAMPS"] = "1"
os.environ.setdefault("DDMI_LIB", os.path.join(ROOT, "diffusiondrive_amd", "_variants", "libddmi_stamps.so"))
from diffusiondrive_amd.config import TransfuserConfig
from diffusiondrive_amd.model import DiffusionDriveModel
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
cfg = TransfuserConfig()
m = DiffusionDriveModel(cfg, seeded_state_dict(cfg, 0), device=0, gemm="f16x3")
B = int(os.environ.get("DDMI_STAMP_B", "64"))
inp = synthetic_inputs(B, 1234)
feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"]).cuda()
for _ in range(4):
    m.forward(feats, noise=nz)
torch.cuda.synchronize()
names = ["qkv", "self_attn", "sa_out", "ln1", "ca_q", "cross_attn", "ca_out", "ln2", "ffn", "ln3"]
LABELS = {1 + 10 * l + i: f"L{l}.{n}" for l in range(3) for i, n in enumerate(names)}
LABELS.update({31: "agent_kv", 32: "ego"})
st = m.tap("tf_stamps").cpu().numpy().view(np.uint64)[: B * 40].reshape(B, 40).astype(np.int64)
live = [k for k in range(40) if (st[:, k] > 0).all()]
parts = []
for a_, b_ in zip(live[:-1], live[1:]):
    parts.append(f"{LABELS.get(b_, b_)}={int(np.median(st[:, b_] - st[:, a_]))}")
tot = int(np.median(st[:, live[-1]] - st[:, live[0]]))
print(f"tfdec total {tot}:\n  " + "\n  ".join(parts), flush=True)
