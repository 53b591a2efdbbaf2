"""GPU diagnostics: per-phase shader-clock stamps of the decoder megakernel (DDMI_MK_STAMPS=1), B = 64."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["DDMI_MK_STAMPS"] = "1"
os.environ.setdefault("DDMI_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "diffusiondrive_amd", "_variants", "libddmi_stamps.so"))
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
LABELS = {1: "pts", 2: "emb", 3: "pa0", 4: "ln+pa3", 6: "logits+sample", 7: "outp", 8: "ag_q", 9: "kv",
          10: "qload", 11: "scores", 12: "pv", 13: "split", 14: "ag_out", 15: "ln12", 24: "ffn_epi", 25: "ln3",
          26: "c0r0", 27: "lnc2", 28: "c3r2", 30: "heads", 31: "final+ddim", 32: "end"}
LABELS.update({16 + 2 * c + h: f"ffn{c}{'ab'[h]}" for c in range(4) for h in range(2)})
for s in range(2):
    for l in range(2):
        st = m.tap(f"mk_stamps_s{s}l{l}").cpu().numpy().view(np.uint64)[: B * 40].reshape(B, 40).astype(np.int64)
        live = [k for k in range(40) if (st[:, k] > 0).all()]
        parts = []
        for a_, b_ in zip(live[:-1], live[1:]):
            parts.append(f"{LABELS.get(b_, b_)}={int(np.median(st[:, b_] - st[:, a_]))}")
        tot = int(np.median(st[:, live[-1]] - st[:, live[0]]))
        print(f"s{s}l{l} total {tot}: " + " ".join(parts), flush=True)
