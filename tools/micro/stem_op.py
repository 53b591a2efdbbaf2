#!/usr/bin/env python3
"""The fused camera stem (dd_op_stem_pool, f16x3) at the bench shape (B = 64, 256 x 1024 x 4), a few launches:
a driver for rocprofv3 PMC passes on stem_pool_kernel (DDMI_LIB selects a library build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
B, H, W = 64, 256, 1024
g = torch.Generator().manual_seed(0)
x = torch.rand(B, H, W, 4, generator=g)
x[..., 3] = 0
x = x.cuda()
w = (torch.randn(64, 7, 7, 4, generator=g) * 0.07).cuda()
b = (torch.randn(64, generator=g) * 0.1).cuda()
out = torch.empty(B, 64, 256, 64, device="cuda")
flags = torch.zeros(1, dtype=torch.int32, device="cuda")
for _ in range(int(os.environ.get("REPS", "4"))):
    _lib.check(lib.dd_op_stem_pool(x.data_ptr(), B, H, W, w.data_ptr(), b.data_ptr(), out.data_ptr(), 0,
                                   flags.data_ptr(), None), lib, op=True)
torch.cuda.synchronize()
print("ok", float(out.abs().mean()))
