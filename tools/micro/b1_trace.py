#!/usr/bin/env python3
"""Batch-1 forwards for a kernel trace (rocprofv3 --kernel-trace -- python tools/micro/b1_trace.py): warm-up, then
N forwards of one scene on a default handle, each followed by a synchronize and a 2 ms host pause, so the trace
splits into forwards at the gaps (tools/micro/b1_timeline.py reads it).

    DDMI_TRACE_B (default 1), DDMI_TRACE_N (default 10), DDMI_TRACE_STREAMS (default: the handle's default)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402

B = int(os.environ.get("DDMI_TRACE_B", "1"))
N = int(os.environ.get("DDMI_TRACE_N", "10"))
cfg = TransfuserConfig()
m = DiffusionDriveModel(cfg, seeded_state_dict(cfg, 0), device=0, gemm=os.environ.get("DDMI_TRACE_GEMM", "f16x3"))
if os.environ.get("DDMI_TRACE_STREAMS"):
    m.set_streams(int(os.environ["DDMI_TRACE_STREAMS"]))
inp = synthetic_inputs(B, 1234, cfg)
feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
nz = torch.from_numpy(inp["noise"]).cuda()
for _ in range(5):
    m.forward(feats, noise=nz)
torch.cuda.synchronize()
t = []
for _ in range(N):
    time.sleep(0.002)
    t0 = time.perf_counter()
    m.forward(feats, noise=nz)
    torch.cuda.synchronize()
    t.append((time.perf_counter() - t0) * 1e3)
t.sort()
print(f"b1_trace: B={B} streams={m.stream_count()} wall ms median {t[len(t) // 2]:.3f} min {t[0]:.3f}", flush=True)
