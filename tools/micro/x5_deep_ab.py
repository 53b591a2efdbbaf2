#!/usr/bin/env python3
"""Same-box A/B of conv_x5's deep-ring form (DDMI_X5_DEEP=1: 16-deep K chunks, 4 stages at 256 x 256) against
the 32-deep 2-stage form, on the shapes the forward routes to 256 x 256 tiles (GPT GEMMs at M = 64 x 320 tokens,
the stride-2 3x3 convs), and checks bit-identity. The op entry point splits the weights on the host per call, so
time it under rocprofv3 (the two forms are separate kernel instances). GPU only.

    rocprofv3 --kernel-trace --stats -d gpurun_out/x5deep -- python tools/micro/x5_deep_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()


def run(x, w, b, res, out, N, H, W, k, s, p, reps):
    B_, _, _, C = x.shape
    for _ in range(reps):
        _lib.check(lib.dd_op_conv2d_x3(x.data_ptr(), B_, H, W, C, w.data_ptr(), b.data_ptr(),
                                       res.data_ptr() if res is not None else None, out.data_ptr(), N, k, k, s, p,
                                       0, 0, None, None), lib, op=True)


def case(name, B_, H, W, C, N, k, s, res_on):
    g = torch.Generator(device="cuda").manual_seed(0)
    p = k // 2
    x = torch.randn(B_, H, W, C, device="cuda", generator=g)
    w = torch.randn(N, k, k, C, device="cuda", generator=g) / (k * k * C) ** 0.5
    b = torch.randn(N, device="cuda", generator=g)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    res = torch.randn(B_, Ho, Wo, N, device="cuda", generator=g) if res_on else None
    outs = {}
    for mode in ("0", "1"):
        os.environ["DDMI_X5_DEEP"] = mode
        out = torch.empty(B_, Ho, Wo, N, device="cuda")
        run(x, w, b, res, out, N, H, W, k, s, p, 10)
        torch.cuda.synchronize()
        outs[mode] = (out, lib.dd_op_last_kernel().decode())
    same = torch.equal(outs["0"][0], outs["1"][0])
    print(f"{name:28s} [{outs['0'][1]}] vs [{outs['1'][1]}]  bit-identical {same}", flush=True)
    return same


ok = True
ok &= case("mlp-up C512 (2048,512)", 64, 320, 1, 512, 2048, 1, 1, False)
ok &= case("mlp-down C512 (512,2048)", 64, 320, 1, 2048, 512, 1, 1, True)
ok &= case("qkv C512 (1536,512)", 64, 320, 1, 512, 1536, 1, 1, False)
ok &= case("qkv C256 (768,256)", 64, 320, 1, 256, 768, 1, 1, False)
ok &= case("mlp-down C256 (256,1024)", 64, 320, 1, 1024, 256, 1, 1, True)
ok &= case("img l3.0 s2 3x3 (256,128)", 64, 32, 128, 128, 256, 3, 2, False)
ok &= case("ragged M (2048,512)", 3, 97, 1, 512, 2048, 1, 1, True)
print("ALL BIT-IDENTICAL" if ok else "MISMATCH", flush=True)
sys.exit(0 if ok else 1)
