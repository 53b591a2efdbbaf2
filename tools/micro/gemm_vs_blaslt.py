#!/usr/bin/env python3
"""How far the GPT-shaped f16x3 GEMMs (M = 64 scenes x 320 tokens, routed to conv_x5 / conv_x3 by
dd_op_conv2d_x3) sit from the vendor library: each shape timed with HIP events (20 reps) beside torch's
fp16 GEMM (hipBLASLt) at K' = 3K - the same f16 products an f16x3 GEMM issues ([ah | ah | al] x [bh; bl; bh]),
fp32 accumulate. dd_op_conv2d_x3 splits the weights on the host per call, so its kernel time comes from the
rocprofv3 kernel trace this script runs under (the event column for it includes host gaps); torch.mm's from events.""" 
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
M = 20480
REPS = 20


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS * 1e3


print(f"{'N':>5} {'K':>5} {'ours_us':>9} {'ours_TF':>8} {'blaslt3K_us':>11} {'blaslt_TF':>9}", flush=True)
for (N, K) in [(1536, 512), (512, 512), (2048, 512), (512, 2048), (768, 256), (256, 256), (1024, 256), (256, 1024)]:
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    c = torch.empty(M, N, device="cuda")

    def ours():
        _lib.check(lib.dd_op_conv2d_x3(a.data_ptr(), 1, M, 1, K, w.data_ptr(), b.data_ptr(), None, c.data_ptr(), N,
                                       1, 1, 1, 0, 0, 0, None, None), lib, op=True)

    a3 = torch.randn(M, 3 * K, device="cuda", dtype=torch.float16)
    w3 = torch.randn(3 * K, N, device="cuda", dtype=torch.float16)
    c3 = torch.empty(M, N, device="cuda", dtype=torch.float16)

    def blaslt():
        torch.mm(a3, w3, out=c3)

    t0 = timed(ours)
    t1 = timed(blaslt)
    fl = 2.0 * M * N * K
    print(f"{N:5d} {K:5d} {t0:9.1f} {fl / t0 / 1e6:8.1f} {t1:11.1f} {fl / t1 / 1e6:9.1f}", flush=True)
print("done", flush=True)
