#!/usr/bin/env python3
"""Microbenchmark of small GEMMs through dd_op_gemm (decoder / tf-decoder shapes); run under
rocprofv3 --kernel-trace --stats for per-kernel device time (DDMI_GEMM_LAT=0/1 picks the kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
SHAPES = [(1280, 256, 256), (1280, 1024, 256), (1280, 256, 1024), (1984, 256, 256), (4096, 512, 512), (1, 1024, 256)]
for M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    c = torch.empty(M, N, device="cuda")
    for _ in range(20):
        _lib.check(lib.dd_op_gemm(a.data_ptr(), M, K, w.data_ptr(), b.data_ptr(), None, c.data_ptr(), N, 0, None),
                   lib, op=True)
    torch.cuda.synchronize()
print("done", flush=True)
