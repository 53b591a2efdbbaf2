#!/usr/bin/env python3
"""Bit-identity A/B of the whole forward between two library builds: the seeded model (seeded_state_dict(cfg, 0)),
f16x3, B = 64 synthetic scenes (seed 1234) with the library DDMI_LIB points at; saves sha256 digests of the trajectory
and of every decoder layer's gathered value rows (taps value_rows_s*l*) to OUT (json); with REF=<json of the other
build> compares them. Also prints the value_proj launch time from the runtime's profiling stats."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402

B = 64
m = DiffusionDriveModel(state_dict=seeded_state_dict(TransfuserConfig(), 0), device=0, gemm="f16x3")
inp = synthetic_inputs(B, 1234)
feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"])
m.forward(feats, noise=nz)
m.set_profiling(True)
m.reset_stats()
for _ in range(5):
    out = m.forward(feats, noise=nz)["trajectory"].numpy()
st = m.kernel_stats("value_proj")
m.set_profiling(False)
assert m.numerics_flags() == 0
res = {"trajectory": hashlib.sha256(out.tobytes()).hexdigest()}
for s in range(2):
    for l in range(2):
        res[f"value_rows_s{s}l{l}"] = hashlib.sha256(m.tap(f"value_rows_s{s}l{l}").cpu().numpy().tobytes()).hexdigest()
print("value_proj", json.dumps(st), flush=True)
json.dump(res, open(os.environ["OUT"], "w"))
if os.environ.get("REF"):
    ref = json.load(open(os.environ["REF"]))
    for k, v in res.items():
        print(f"{k}: bit-identical {v == ref[k]}", flush=True)
    assert all(v == ref[k] for k, v in res.items())
m.close()
print("model_ab done", flush=True)
