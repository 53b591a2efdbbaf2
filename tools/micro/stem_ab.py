#!/usr/bin/env python3
"""Bit-identity and timing A/B of the fused stems between two library builds: runs both stems (camera NCHW 3 x 256 x
1024 and LiDAR 1 x 256 x 256 at B = 64, f16x3 and bf16) with the library DDMI_LIB points at, saves the pooled maps'
sha256 digests to OUT (json; the maps themselves are 268 MB); with REF=<json of the other build> compares them. Timing:
run under rocprofv3 --kernel-trace."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
B = 64
res = {}
g = torch.Generator().manual_seed(0)
for C, H, W in ((3, 256, 1024), (1, 256, 256)):
    x = torch.rand(B, C, H, W, generator=g).cuda()
    w = torch.randn(64, 7, 7, 4, generator=g) * 0.07
    w[..., C:] = 0
    w = w.cuda()
    b = (torch.randn(64, generator=g) * 0.1).cuda()
    for prec in (0, 1):
        out = torch.empty(B, H // 4, W // 4, 64, device="cuda")
        flags = torch.zeros(1, dtype=torch.int32, device="cuda")
        for _ in range(int(os.environ.get("REPS", "10"))):
            _lib.check(lib.dd_op_stem_pool_nchw(x.data_ptr(), B, C, H, W, w.data_ptr(), b.data_ptr(), out.data_ptr(),
                                                prec, flags.data_ptr(), None), lib, op=True)
        torch.cuda.synchronize()
        assert int(flags.item()) == 0, "numerics flag"
        res[f"C{C}_p{prec}"] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
json.dump(res, open(os.environ["OUT"], "w"))
if os.environ.get("REF"):
    ref = json.load(open(os.environ["REF"]))
    for k, v in res.items():
        print(f"{k}: bit-identical {v == ref[k]}", flush=True)
        assert v == ref[k], k
print("stem_ab done", flush=True)
