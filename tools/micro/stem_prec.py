#!/usr/bin/env python3
"""Precision of the fused stem forms against fp64 (GPU): the 4-channel-pixel form (DDMI_STEM1=0, K = 224) and the
one-channel LiDAR form (DDMI_STEM1=1, K = 64, f16x3 cross products in an accumulator of their own). Round 6 ran it
with a third form, the one-channel form with one accumulator (profiles/round6_stem1.md). Inputs: a LiDAR-like histogram (multiples of 0.2, ~90 % zeros) and dense |N(0,1)|; seeded weights.
Prints max / mean abs error over the pooled map, relative to max |ref|, and the bias (mean signed error)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(5)
B, H, W = 8, 256, 256
lid = (torch.randint(1, 6, (B, 1, H, W), generator=g).float() / 5) * (torch.rand(B, 1, H, W, generator=g) < 0.1).float()
dense = torch.randn(B, 1, H, W, generator=g).abs()
w = torch.randn(64, 4, 7, 7, generator=g) / np.sqrt(49)
w[:, 1:] = 0
b = torch.randn(64, generator=g) * 0.1
for name, x in (("lidar", lid), ("dense", dense)):
    ref = F.max_pool2d(F.relu(F.conv2d(x.double(), w[:, :1].double(), b.double(), 2, 3)), 3, 2, 1)
    scale = float(ref.abs().max())
    for form in ("0", "1"):
        os.environ["DDMI_STEM1"] = form
        out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        xin, win, bin_ = x.to(dev), w.permute(0, 2, 3, 1).contiguous().to(dev), b.to(dev)
        _lib.check(lib.dd_op_stem_pool_nchw(xin.data_ptr(), B, 1, H, W, win.data_ptr(), bin_.data_ptr(),
                                             out.data_ptr(), 0, flags.data_ptr(), None), lib)
        torch.cuda.synchronize()
        d = out.permute(0, 3, 1, 2).double().cpu() - ref
        print(f"{name:5s} DDMI_STEM1={form}: max abs err / max|ref| {float(d.abs().max()) / scale:.3e}  "
              f"mean abs {float(d.abs().mean()) / scale:.3e}  mean signed {float(d.mean()) / scale:+.3e}  "
              f"flags {int(flags.item())}", flush=True)
