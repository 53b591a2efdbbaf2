#!/usr/bin/env python3
"""The tf decoder at one batch three ways - four workgroups per scene, one workgroup (DDMI_TF_GROUPS=1), the unfused
chain (DDMI_TFDEC_MK=0) - and the pairwise max differences of query_out (with where the largest sits). GPU only.

    TF3_B=16 python tools/debug/tf_three.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402

B = int(os.environ.get("TF3_B", "16"))
sd = seeded_state_dict(TransfuserConfig(), 0)
inp = synthetic_inputs(B, 43)
f = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
q = {}
for name, env in (("g4", {"DDMI_TF_GROUPS": "4"}), ("g1", {"DDMI_TF_GROUPS": "1"}), ("unfused", {"DDMI_TFDEC_MK": "0"})):
    for k in ("DDMI_TF_GROUPS", "DDMI_TFDEC_MK"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = DiffusionDriveModel(state_dict=sd, device=0, gemm="f16x3")
    m.forward(f, noise=torch.from_numpy(inp["noise"]))
    q[name] = m.tap("query_out").cpu().numpy()[: B * 31 * 256].reshape(B, 31, 256).copy()
    m.close()
for a, b in (("g4", "g1"), ("g4", "unfused"), ("g1", "unfused")):
    d = np.abs(q[a] - q[b])
    i = np.unravel_index(int(d.argmax()), d.shape)
    per_scene = d.max(axis=(1, 2))
    print(f"B={B} {a} vs {b}: max {d.max():.3e} at scene/query/ch {i}; per-scene max {np.round(per_scene * 1e5, 1)} e-5",
          flush=True)
