#!/usr/bin/env python3
"""Both fused stems on the reference's NCHW tensors at the bench shape (B = 64: camera 3 x 256 x 1024, LiDAR
1 x 256 x 256) through dd_op_stem_pool_nchw, REPS launches each: run under rocprofv3 --kernel-trace --stats for the
per-kernel averages (DDMI_STEM_DIAG splits the phases; DDMI_LIB selects a library build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
B = 64
prec = int(os.environ.get("PREC", "0"))
g = torch.Generator().manual_seed(0)
for C, H, W in ((3, 256, 1024), (1, 256, 256)):
    x = torch.rand(B, C, H, W, generator=g).cuda()
    w = torch.randn(64, 7, 7, 4, generator=g) * 0.07
    w[..., C:] = 0
    w = w.cuda()
    b = (torch.randn(64, generator=g) * 0.1).cuda()
    out = torch.empty(B, H // 4, W // 4, 64, device="cuda")
    flags = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(int(os.environ.get("REPS", "6"))):
        _lib.check(lib.dd_op_stem_pool_nchw(x.data_ptr(), B, C, H, W, w.data_ptr(), b.data_ptr(), out.data_ptr(), prec,
                                            flags.data_ptr(), None), lib, op=True)
    torch.cuda.synchronize()
    print(f"stem C={C}: ok {float(out.abs().mean()):.6f}")
