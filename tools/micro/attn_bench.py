#!/usr/bin/env python3
"""Microbenchmark of the fused GPT attention op (dd_op_gpt_attention) at the bench shapes (B=64, T=320)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
B, T = 64, 320
PREC = int(os.environ.get("ATTN_PREC", "1"))  # 1: the f16x3 kernel (default mode), 0: fp32 MFMA
for C in (64, 128, 256, 512):
    qkv = torch.randn(B, T, 3 * C, device="cuda")
    y = torch.empty(B, T, C, device="cuda")
    for _ in range(3):
        _lib.check(lib.dd_op_gpt_attention(qkv.data_ptr(), y.data_ptr(), B, T, C, 4, PREC, None), lib, op=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        lib.dd_op_gpt_attention(qkv.data_ptr(), y.data_ptr(), B, T, C, 4, PREC, None)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    fl = 4.0 * B * T * T * C
    # float64 reference on 4 scenes: max |err| / max |y|
    hs = C // 4
    x = qkv[:4].double().view(4, T, 3, 4, hs)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    ref = torch.softmax(q @ k.transpose(-1, -2) / hs ** 0.5, -1) @ v
    ref = ref.transpose(1, 2).reshape(4, T, C)
    err = ((y[:4].double() - ref).abs().max() / ref.abs().max()).item()
    print(f"C={C:4d} hs={hs:3d}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s  rel err {err:.2e}", flush=True)
