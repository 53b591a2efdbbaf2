#!/usr/bin/env python3
"""Where a union-staged value_proj workgroup's time goes (diagnostic build DDMI_BUILD_VARIANT=vust): per-workgroup
shader-clock stamps at start / K loop entry / K loop exit / end and wave 0's cycles inside the step barriers and the
union-store waits, for the last value_proj launch of a B = 64 forward (median and spread over the workgroups)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("DDMI_LIB", os.path.join(ROOT, "diffusiondrive_amd", "_variants", "libddmi_vust.so"))
from diffusiondrive_amd import _lib  # noqa: E402
from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402

cfg = TransfuserConfig()
m = DiffusionDriveModel(cfg, seeded_state_dict(cfg, 0), device=0, gemm="f16x3")
B = int(os.environ.get("DDMI_STAMP_B", "64"))
inp = synthetic_inputs(B, 1234)
feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"]).cuda()
lib = _lib.load()
rd = lib.dd_vu_stamps_read
rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
rd.restype = ctypes.c_int
N = 8192 * 6
buf = np.zeros(N, dtype=np.uint64)
for it in range(3):
    m.forward(feats, noise=nz)
    torch.cuda.synchronize()
    assert rd(buf.ctypes.data, N) == 0
    st = buf.reshape(8192, 6).astype(np.int64)
    live = st[st[:, 0] > 0]
    pro, kl, epi = live[:, 1] - live[:, 0], live[:, 2] - live[:, 1], live[:, 3] - live[:, 2]
    tot = live[:, 3] - live[:, 0]
    span = live[:, 3].max() - live[:, 0].min()
    q = lambda x: f"{int(np.median(x))} [{int(np.percentile(x, 10))}..{int(np.percentile(x, 90))}]"
    print(f"forward {it}: {len(live)} workgroups, launch span {span} ticks; per workgroup: prologue {q(pro)}, "
          f"K loop {q(kl)}, epilogue {q(epi)}, total {q(tot)}; wave 0 in step barriers {q(live[:, 4])}, "
          f"in union-store waits {q(live[:, 5])}; start skew {int(live[:, 0].max() - live[:, 0].min())}", flush=True)
