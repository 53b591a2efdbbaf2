#!/usr/bin/env python3
"""The GPT-shaped f16x3 GEMMs (M = 20480) through dd_op_conv2d_x3, REPS launches per shape, for A/Bs of conv_x5 forms
under rocprofv3 --kernel-trace; `--parse <trace dir>` prints the per-shape kernel averages (launches in shape order,
the first 3 of each shape dropped) and checks nothing else. Shapes: (N, K) of the C = 512 / 256 blocks."""
import csv
import glob
import os
import sys

SHAPES = [(128, 512), (256, 256), (128, 128), (64, 256), (256, 64), (64, 64), (192, 64), (512, 128), (384, 128)]
REPS = 13

if "--parse" in sys.argv:
    d = sys.argv[sys.argv.index("--parse") + 1]
    f = glob.glob(f"{d}/**/*_kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows
           if "conv_x" in r["Kernel_Name"]]
    for i, (N, K) in enumerate(SHAPES):
        s = seq[i * REPS:(i + 1) * REPS]
        avg = sum(t for _, t in s[3:]) / (REPS - 3)
        name = s[0][0].split("(")[0].replace("void ddmi::", "")
        print(f"N {N:5d} K {K:5d}  {avg:8.1f} us  {2.0 * 20480 * N * K / avg / 1e6:6.1f} TF  {name}")
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from diffusiondrive_amd import _lib  # noqa: E402

lib = _lib.load()
M = 20480
for (N, K) in SHAPES:
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    c = torch.empty(M, N, device="cuda")
    ref = None
    for _ in range(REPS):
        _lib.check(lib.dd_op_conv2d_x3(a.data_ptr(), 1, M, 1, K, w.data_ptr(), b.data_ptr(), None, c.data_ptr(), N,
                                       1, 1, 1, 0, 0, 0, None, None), lib, op=True)
    torch.cuda.synchronize()
    r = a.double() @ w.double().T + b.double()
    err = float(((c.double() - r).abs().max() / r.abs().max()))
    print(f"N {N} K {K} max rel err {err:.2e}", flush=True)
    assert err < 1e-5
print("done", flush=True)
