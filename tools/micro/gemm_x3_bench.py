#!/usr/bin/env python3
"""Microbenchmark of the GPT-shaped f16x3 GEMMs (M = 64 scenes x 320 tokens) through dd_op_conv2d_x3
as 1x1 convs; run under rocprofv3 --kernel-trace --stats. Cases: with / without the in-place residual."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
M = 20480
for (N, K, res) in [(512, 512, False), (512, 512, True), (512, 2048, False), (512, 2048, True), (2048, 512, False),
                    (256, 256, False), (256, 256, True), (1536, 512, False)]:
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    c = torch.randn(M, N, device="cuda")
    for _ in range(10):
        _lib.check(lib.dd_op_conv2d_x3(a.data_ptr(), 1, M, 1, K, w.data_ptr(), b.data_ptr(),
                                       c.data_ptr() if res else None, c.data_ptr(), N, 1, 1, 1, 0, 0, 0, None, None),
                   lib, op=True)
    torch.cuda.synchronize()
    print(N, K, res, flush=True)
print("done", flush=True)
