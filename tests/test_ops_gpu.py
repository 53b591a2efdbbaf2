"""Per-kernel parity on the GPU: each ddmi kernel (called through the C ABI) vs a plain
PyTorch-CPU fp32 reference of the same op on the same seeded inputs.

Tolerances: fp32 MFMA is an exact fp32 fma chain that differs from the CPU only in summation
order -> relative error ~1e-6 of sum|a*b|; we assert max|err| <= 2e-5 * (1 + max|ref|) for
contractions and 1e-5 for elementwise / reduction kernels.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from diffusiondrive_amd import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def g(t):
    """Device copy. Callers must keep the returned tensor alive until the op has run: a temporary
    passed as ``g(x).data_ptr()`` is freed (and its memory reused) before the kernel executes."""
    return t.to(DEV).contiguous()


def rnd(*shape, seed=0, scale=1.0):
    gen = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=gen) * scale


def ok(rc, lib):
    _lib.check(rc, lib, op=True)
    torch.cuda.synchronize()


def close(a, ref, tol):
    a = a.detach().cpu().double()
    ref = ref.detach().cpu().double()
    err = (a - ref).abs().max().item()
    lim = tol * (1.0 + ref.abs().max().item())
    assert err <= lim, f"max err {err:.3e} > {lim:.3e}"
    return err


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s,p,relu,res", [
    (2, 16, 24, 64, 64, 3, 1, 1, True, True),     # BasicBlock conv2 (+residual)
    (2, 16, 24, 64, 128, 3, 2, 1, True, False),   # stage-entry conv1 (stride 2)
    (2, 16, 24, 64, 128, 1, 2, 0, False, False),  # downsample 1x1/s2
    (1, 40, 70, 4, 64, 7, 2, 3, True, False),     # stem (3 -> padded 4 channels)
    (2, 8, 8, 512, 7, 1, 1, 0, False, False),     # tiny Cout (semantic logits)
    (1, 64, 64, 256, 256, 3, 1, 1, True, False),  # value_proj
    (3, 5, 7, 320, 40, 1, 1, 0, True, True),      # ragged M / N
])
def test_conv2d(gpu, B, H, W, Cin, Cout, k, s, p, relu, res):
    x = rnd(B, Cin, H, W, seed=1)
    w = rnd(Cout, Cin, k, k, seed=2, scale=1.0 / np.sqrt(Cin * k * k))
    b = rnd(Cout, seed=3)
    ref = F.conv2d(x, w, b, s, p)
    r = rnd(*ref.shape, seed=4) if res else None
    if res:
        ref = ref + r
    if relu:
        ref = F.relu(ref)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    xin, win, bin_ = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b)
    rin = g(r.permute(0, 2, 3, 1)) if res else None
    ok(gpu.dd_op_conv2d(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(),
                        rin.data_ptr() if res else None, out.data_ptr(), Cout, k, k, s, p, int(relu), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 2e-5)


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s,p,relu,res", [
    (2, 16, 24, 64, 64, 3, 1, 1, True, True),     # BasicBlock conv2 (+residual), Cin % 32 == 0 path
    (2, 16, 24, 64, 128, 3, 2, 1, True, False),   # stage-entry conv1 (stride 2)
    (2, 16, 24, 64, 128, 1, 2, 0, False, False),  # downsample 1x1/s2
    (1, 40, 70, 4, 64, 7, 2, 3, True, False),     # stem (3 -> padded 4 channels), generic K path
    (2, 8, 8, 512, 7, 1, 1, 0, False, False),     # tiny Cout
    (1, 64, 64, 256, 256, 3, 1, 1, True, False),  # value_proj
    (3, 5, 7, 320, 40, 1, 1, 0, True, True),      # ragged M / N
    (2, 64, 80, 64, 64, 3, 1, 1, True, False),    # Cout 64, 256-row tiles
    (1, 48, 64, 128, 256, 3, 1, 1, False, True),  # 128x128 tiles
    (1, 9, 11, 36, 24, 3, 1, 1, False, False),    # Cin % 32 != 0, K tail
    # grids that fill the chip take the LDS-DMA kernel (conv_x5.hip)
    (16, 64, 64, 64, 64, 3, 1, 1, True, True),    # 256 x 64 tiles, tap walk, padding via OOB DMA
    (4, 128, 128, 32, 128, 3, 1, 1, True, False), # 256 x 128 tiles, Cin = 32
    (1, 256, 256, 128, 256, 1, 1, 0, False, True),# 256 x 256 tiles, 1x1
    (16, 64, 64, 36, 200, 3, 1, 1, True, False),  # generic K path, ragged N in a 256-wide tile
    (1, 518, 518, 4, 64, 7, 2, 3, True, False),   # stem geometry (7x7/s2 on 4 padded channels)
    (3, 90, 250, 64, 256, 3, 2, 1, False, False), # stride 2, ragged M
    (1, 128, 128, 64, 512, 1, 1, 0, True, True),  # 256 x 128 tiles (3 stages) for Cout > 128
    (1, 64, 128, 128, 512, 1, 1, 0, False, True), # 128 x 128 tiles (4 waves, 3 stages)
    (1, 70, 130, 160, 400, 1, 1, 0, False, True), # 128 x 128 tiles, ragged M and N
    (1, 64, 128, 132, 512, 1, 1, 0, True, False), # 128 x 128 tiles, generic K (Cin % 32 != 0)
    (1, 256, 256, 64, 256, 3, 2, 1, True, False), # 128 x 128 tiles, 3x3 stride-2 tap walk
    (4, 130, 126, 64, 128, 1, 2, 0, False, False),# 1x1 stride-2 downsample, 128 x 128 two per CU, ragged M
    (1, 161, 128, 256, 1024, 1, 1, 0, True, False),# GPT MLP-up shape (C = 256), 128 x 128 two per CU, ragged M
    # 3x3 / stride 1 convs take the halo-reuse direct kernel (conv_x6.hip)
    (2, 8, 40, 128, 192, 3, 1, 1, True, True),    # 8 x 32 tiles, ragged W, BN 64 x 3
    (1, 12, 70, 64, 100, 3, 1, 1, False, True),   # 8 x 32 tiles ragged in H and W, ragged N
    (1, 20, 20, 96, 36, 3, 1, 1, True, False),    # 16 x 16 tiles ragged, Cout < BN
    (8, 64, 64, 32, 200, 3, 1, 1, True, True),    # BN 128 ring (256 workgroups), ragged N
    (64, 16, 16, 256, 256, 3, 1, 1, True, True),  # LiDAR layer3 shape
])
def test_conv2d_f16x3(gpu, B, H, W, Cin, Cout, k, s, p, relu, res):
    """f16x3 split-MFMA conv vs PyTorch-CPU fp32 (tolerance: fp32-class, 3e-5 of max|ref|)."""
    x = rnd(B, Cin, H, W, seed=11)
    w = rnd(Cout, Cin, k, k, seed=12, scale=1.0 / np.sqrt(Cin * k * k))
    b = rnd(Cout, seed=13)
    ref = F.conv2d(x.double(), w.double(), b.double(), s, p)
    r = rnd(*ref.shape, seed=14) if res else None
    if res:
        ref = ref + r.double()
    if relu:
        ref = F.relu(ref)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win, bin_ = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b)
    rin = g(r.permute(0, 2, 3, 1)) if res else None
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(),
                           rin.data_ptr() if res else None, out.data_ptr(), Cout, k, k, s, p, int(relu), 0,
                           flags.data_ptr(), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 3e-5)
    assert int(flags.item()) == 0
    # bf16 (reduced precision, one product): same kernel family, bf16-rounding tolerance
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(),
                           rin.data_ptr() if res else None, out.data_ptr(), Cout, k, k, s, p, int(relu), 1,
                           flags.data_ptr(), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 3e-2)


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s,p,relu,res,route", [
    # the batch-dependent routes the B = 64 benchmark forward takes (bench.py's workload)
    (64, 8, 32, 512, 512, 3, 1, 1, True, True, "conv_x6<8,32,128,4,2>"),     # image layer4 (256 WGs of BN 128)
    (64, 32, 128, 128, 128, 3, 1, 1, True, True, "conv_x6<16,16,128,4,2>"),  # image layer2 3x3
    (64, 64, 256, 64, 64, 3, 1, 1, True, True, "conv_x6<16,16,64,4,1>"),     # image layer1 (4-wave, 2 WG / CU)
    (64, 64, 256, 64, 128, 3, 2, 1, True, False, "conv_x5<128,128>"),        # image layer2 entry, 3x3 / s2 (2 WG / CU)
    (64, 32, 128, 128, 256, 3, 2, 1, True, False, "conv_x5<256,256>"),       # image layer3 entry, 3x3 / s2
    (1, 160, 128, 512, 2048, 1, 1, 0, True, False, "conv_x5<128,128>"),      # GPT MLP-up at C = 512 (M = 20480)
    (1, 160, 128, 2048, 512, 1, 1, 0, False, True, "conv_x5<128,128>"),      # GPT MLP-down at C = 512 (640 tiles)
    (1, 160, 128, 256, 768, 1, 1, 0, False, False, "conv_x5<256,256>"),      # GPT qkv at C = 256 (240 tiles)
    (1, 160, 128, 128, 384, 1, 1, 0, False, False, "conv_x5<256,128>"),      # GPT qkv at C = 128
    (1, 160, 128, 256, 256, 1, 1, 0, False, True, "conv_x3<64,64,f16x3>"),   # GPT proj at C = 256 (80 tiles)
    (64, 8, 8, 512, 512, 3, 1, 1, True, True, "conv_x6<8,8,128,2,4>"),       # LiDAR layer4 (8 x 8 maps)
    (2, 8, 8, 512, 512, 3, 1, 1, True, True, "conv_x3<64,64,f16x3,ksplit>"), # too few 8 x 8 tiles for conv_x6
])
def test_conv2d_f16x3_b64_routes(gpu, B, H, W, Cin, Cout, k, s, p, relu, res, route):
    """f16x3 conv at the B = 64 forward's shapes: the dispatcher must take the named kernel / tile
    configuration (dd_op_last_kernel) and match PyTorch-CPU fp64 to 3e-5 of max|ref|."""
    x = rnd(B, Cin, H, W, seed=61)
    w = rnd(Cout, Cin, k, k, seed=62, scale=1.0 / np.sqrt(Cin * k * k))
    b = rnd(Cout, seed=63)
    ref = F.conv2d(x.double(), w.double(), b.double(), s, p)
    r = rnd(*ref.shape, seed=64) if res else None
    if res:
        ref = ref + r.double()
    if relu:
        ref = F.relu(ref)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win, bin_ = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b)
    rin = g(r.permute(0, 2, 3, 1)) if res else None
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(),
                           rin.data_ptr() if res else None, out.data_ptr(), Cout, k, k, s, p, int(relu), 0,
                           flags.data_ptr(), None), gpu)
    assert gpu.dd_op_last_kernel().decode() == route
    close(out.permute(0, 3, 1, 2), ref, 3e-5)
    assert int(flags.item()) == 0


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("B,H,W,Cin,Cout", [
    (1, 8, 32, 512, 512),    # image layer 4 at batch 1
    (2, 16, 64, 256, 256),   # image layer 3
    (1, 64, 256, 64, 64),    # image layer 1
    (1, 12, 70, 64, 100),    # ragged H, W and N
])
def test_conv2d_small_grid_form_is_bit_identical(gpu, monkeypatch, B, H, W, Cin, Cout, prec):
    """conv_x6 at small batches: 8 x 8 pixel tiles x 64 channels (4 waves) instead of the routed form, whose grid
    would have fewer than 128 workgroups. Every form walks K in the same order (32-channel chunk, tap, k16 half), so
    the output is bit-identical to the routed form's (DDMI_X6_SMALL=0) and within the f16x3 / bf16 bar of fp64."""
    if prec and Cin % 64:
        pytest.skip("bf16 takes 64-channel chunks")
    x = rnd(B, Cin, H, W, seed=75)
    w = rnd(Cout, Cin, 3, 3, seed=76, scale=1.0 / np.sqrt(Cin * 9))
    b = rnd(Cout, seed=77)
    r = rnd(B, Cout, H, W, seed=78)
    xin, win, bin_, rin = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b), g(r.permute(0, 2, 3, 1))

    monkeypatch.setenv("DDMI_X3_SPLIT", "1")  # conv_x6's forms, not conv_x3's K split ahead of them

    def run(small):
        monkeypatch.setenv("DDMI_X6_SMALL", small)
        out = torch.empty(B, H, W, Cout, device=DEV)
        flags = torch.zeros(1, dtype=torch.int32, device=DEV)
        ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(), rin.data_ptr(),
                               out.data_ptr(), Cout, 3, 3, 1, 1, 1, prec, flags.data_ptr(), None), gpu)
        assert int(flags.item()) == 0
        return out, gpu.dd_op_last_kernel().decode()

    small, route = run("1")
    routed, route0 = run("0")
    assert route.startswith("conv_x6<8,8,64,2,2") and route0 != route, (route, route0)
    assert torch.equal(small, routed)
    if prec == 0:
        ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), 1, 1) + r.double())
        close(small.permute(0, 3, 1, 2), ref, 3e-5)


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s", [
    (1, 8, 8, 512, 512, 3, 1),    # LiDAR layer-4 3x3 at batch 1 (8 tiles, K = 4608: 8 splits)
    (2, 8, 8, 512, 512, 3, 1),    # 16 tiles: 4 splits
    (1, 8, 8, 256, 512, 3, 2),    # layer-4 entry 3x3 / s2 (2 tiles of M = 16)
    (1, 8, 8, 2048, 512, 1, 1),   # 1x1, K = 2048: 8 splits
    (1, 5, 7, 1056, 200, 1, 1),   # ragged M, N (Cout % 64 != 0) and K chunks (33 over 4 splits)
    (1, 8, 32, 512, 512, 3, 1),   # image layer 4 at batch 1: ahead of conv_x6 (32 tiles, 4 splits)
    (1, 16, 16, 256, 256, 3, 1),  # LiDAR layer 3 at batch 1 (16 tiles, 4 splits)
])
def test_conv_x3_k_split(gpu, monkeypatch, B, H, W, Cin, Cout, k, s):
    """conv_x3's K-split form for grids far below the chip (default DDMI_X3_SPLIT=2, ahead of conv_x6; 0 disables;
    read per dispatch):
    S workgroups per tile over disjoint K-chunk ranges, partials summed in split order by the reduce launch, which
    applies bias / residual / ReLU. A different summation order from the one-workgroup form, so the bar is the f16x3
    one against fp64 (both forms), and the split output is the same on every run."""
    p = k // 2
    x = rnd(B, Cin, H, W, seed=91)
    w = rnd(Cout, Cin, k, k, seed=92, scale=1.0 / np.sqrt(Cin * k * k))
    b = rnd(Cout, seed=93)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    r = rnd(B, Cout, Ho, Wo, seed=94)
    xin, win, bin_, rin = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b), g(r.permute(0, 2, 3, 1))

    def run(split):
        monkeypatch.setenv("DDMI_X3_SPLIT", split)
        out = torch.full((B, Ho, Wo, Cout), float("nan"), device=DEV)
        flags = torch.zeros(1, dtype=torch.int32, device=DEV)
        ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(), rin.data_ptr(),
                               out.data_ptr(), Cout, k, k, s, p, 1, 0, flags.data_ptr(), None), gpu)
        assert int(flags.item()) == 0
        return out, gpu.dd_op_last_kernel().decode()

    sp, route = run("2")
    sp2, _ = run("2")
    base, route0 = run("0")
    assert route == "conv_x3<64,64,f16x3,ksplit>" and route0 != route, (route, route0)
    assert torch.equal(sp, sp2)
    ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), s, p) + r.double())
    close(sp.permute(0, 3, 1, 2), ref, 3e-5)
    close(base.permute(0, 3, 1, 2), ref, 3e-5)


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s,p,res,route", [
    (64, 8, 32, 512, 512, 3, 1, 1, True, "conv_x6<8,32,128,4,2,bf16>"),     # image layer4
    (64, 8, 8, 512, 512, 3, 1, 1, True, "conv_x6<8,8,128,2,4,bf16>"),       # LiDAR layer4 (8 x 8 maps)
    (16, 32, 128, 128, 128, 3, 1, 1, True, "conv_x6<16,16,128,4,2,bf16>"),  # layer2 3x3
    (4, 64, 256, 64, 64, 3, 1, 1, False, "conv_x6<16,16,64,4,2,bf16>"),     # layer1 (8-wave BN 64 form)
    (2, 12, 70, 128, 100, 3, 1, 1, True, "conv_x6<8,8,64,2,2,bf16>"),       # ragged H / W / N: a small grid, 8 x 8 tiles
    (1, 160, 128, 512, 2048, 1, 1, 0, False, "conv_x5<256,256,bf16>"),      # GPT MLP-up (M = 20480)
    (64, 64, 256, 64, 256, 1, 1, 0, True, "conv_x5<128,128,bf16>"),         # ResNet-50 layer1 expand 1x1 (2 WG / CU)
    (64, 64, 256, 64, 128, 3, 2, 1, False, "conv_x5<256,128,bf16>"),        # stage entry 3x3 / s2
    (16, 64, 64, 36, 64, 3, 1, 1, False, "conv_x5<256,64,bf16>"),           # generic K (Cin % 32 != 0)
    (3, 5, 7, 320, 40, 1, 1, 0, True, "conv_x3<64,64,bf16>"),               # small grid: register-staged kernel
])
def test_conv2d_bf16(gpu, B, H, W, Cin, Cout, k, s, p, res, route):
    """bf16 mode (configs C2-bf16 / C4): one bf16 product per MAC on the direct 3x3 kernel (64-channel K
    chunks), the LDS-DMA implicit GEMM (A converted at fragment-read time) or conv_x3. Reference: the same
    conv on bf16-rounded operands in fp64 (only the fp32 accumulation order differs), 1e-4 of max|ref|;
    and vs the unrounded conv, bf16 class."""
    x = rnd(B, Cin, H, W, seed=71)
    w = rnd(Cout, Cin, k, k, seed=72, scale=1.0 / np.sqrt(Cin * k * k))
    b = rnd(Cout, seed=73)
    ref0 = F.conv2d(x.double(), w.double(), b.double(), s, p)
    r = rnd(*ref0.shape, seed=74) if res else None
    # the kernels round x to bf16 (RNE) and use the bf16 image of w * 2^e (exact scaling)
    ref_b = F.relu(F.conv2d(x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double(), b.double(), s, p)
                   + (r.double() if res else 0))
    ref = F.relu(ref0 + (r.double() if res else 0))
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win, bin_ = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b)
    rin = g(r.permute(0, 2, 3, 1)) if res else None
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), bin_.data_ptr(),
                           rin.data_ptr() if res else None, out.data_ptr(), Cout, k, k, s, p, 1, 1,
                           flags.data_ptr(), None), gpu)
    assert gpu.dd_op_last_kernel().decode() == route
    close(out.permute(0, 3, 1, 2), ref_b, 1e-4)
    close(out.permute(0, 3, 1, 2), ref, 3e-2)


@pytest.mark.parametrize("B,H,W", [(2, 64, 256), (1, 40, 72), (2, 37, 50)])
def test_stem_pool_bf16(gpu, B, H, W):
    """bf16 fused stem (one bf16 product per MAC) vs PyTorch fp64 on bf16-rounded operands."""
    x = rnd(B, 4, H, W, seed=81).abs()
    x[:, 3] = 0.0
    w = rnd(64, 4, 7, 7, seed=82, scale=1.0 / np.sqrt(196))
    b = rnd(64, seed=83)
    xb, wb = x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double()
    ref = F.max_pool2d(F.relu(F.conv2d(xb, wb, b.double(), 2, 3)), 3, 2, 1)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win, bin_ = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b)
    ok(gpu.dd_op_stem_pool(xin.data_ptr(), B, H, W, win.data_ptr(), bin_.data_ptr(), out.data_ptr(), 1,
                           flags.data_ptr(), None), gpu)
    assert gpu.dd_op_last_kernel().decode() == "stem_pool<bf16>"
    close(out.permute(0, 3, 1, 2), ref, 1e-4)


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("B,C,H,W", [(2, 1, 256, 256), (1, 1, 40, 72), (2, 1, 37, 50), (2, 3, 64, 256), (1, 2, 37, 50)])
@pytest.mark.parametrize("one", [False, True])
def test_stem_pool_nchw(gpu, monkeypatch, B, C, H, W, prec, one):
    """The fused stem on the caller's NCHW tensor (C = 1..3 as 4-channel pixels; with DDMI_STEM1=1 the LiDAR
    histogram's opt-in one-channel form, K = 7 x 8 taps in 4 k16 steps from 4 column-shifted copies of the patch) vs
    PyTorch fp64 (bf16: on bf16-rounded operands)."""
    if one and C != 1:
        pytest.skip("the one-channel form takes C = 1")
    monkeypatch.setenv("DDMI_STEM1", "1" if one else "0")
    x = rnd(B, C, H, W, seed=85).abs()
    w = rnd(64, 4, 7, 7, seed=86, scale=1.0 / np.sqrt(49 * C))
    w[:, C:] = 0.0  # taps of the missing channels (their weights are never read on the NCHW path)
    b = rnd(64, seed=87)
    xr, wr = (x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double()) if prec else (x.double(), w.double())
    ref = F.max_pool2d(F.relu(F.conv2d(xr, wr[:, :C], b.double(), 2, 3)), 3, 2, 1)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win, bin_ = g(x), g(w.permute(0, 2, 3, 1)), g(b)
    ok(gpu.dd_op_stem_pool_nchw(xin.data_ptr(), B, C, H, W, win.data_ptr(), bin_.data_ptr(), out.data_ptr(), prec,
                                flags.data_ptr(), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 1e-4 if prec else 3e-5)
    assert int(flags.item()) == 0


@pytest.mark.parametrize("scale", [2.0 ** -6, 2.0 ** -10])
def test_conv2d_f16x3_small_activations(gpu, scale):
    """The f16x3 subnormal-lo regime: activations well below 2^-3 have a lo part below fp16's
    smallest normal (2^-14), rounded to the subnormal spacing 2^-24, i.e. an absolute operand error <= 2^-25 - against
    max|x| = scale that is a relative 2^-25 / scale (2^-19 at 2^-6, 2^-15 at 2^-10). The conv through conv_x6 must stay
    within that bound (x sqrt(K) accumulation headroom) of the fp64 result."""
    B, H, W, Cin, Cout = 2, 32, 32, 64, 64
    x = rnd(B, Cin, H, W, seed=41).abs() * scale
    w = rnd(Cout, Cin, 3, 3, seed=42, scale=1.0 / np.sqrt(Cin * 9))
    ref = F.conv2d(x.double(), w.double(), None, 1, 1)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1))
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), B, H, W, Cin, win.data_ptr(), None, None, out.data_ptr(), Cout, 3, 3, 1,
                           1, 0, 0, flags.data_ptr(), None), gpu)
    assert gpu.dd_op_last_kernel().decode().startswith("conv_x6")
    rel = float((out.permute(0, 3, 1, 2).double().cpu() - ref).abs().max() / ref.abs().max())
    bound = max(3e-5, 2.0 ** -25 / scale * np.sqrt(Cin * 9) / 4)
    print(f"small activations: scale {scale:g} rel {rel:.3g} bound {bound:.3g}")
    assert rel <= bound, (scale, rel, bound)
    assert int(flags.item()) == 0


def test_conv2d_f16x3_flags_overflow(gpu):
    """An activation beyond the fp16 range must raise DD_NUM_F16_OVERFLOW_BIT (never pass silently)."""
    x = rnd(1, 32, 8, 8, seed=15)
    x[0, 3, 2, 2] = 1e6
    w = rnd(32, 32, 1, 1, seed=16)
    out = torch.empty(1, 8, 8, 32, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1))
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), 1, 8, 8, 32, win.data_ptr(), None, None, out.data_ptr(), 32, 1, 1, 1, 0,
                           0, 0, flags.data_ptr(), None), gpu)
    assert int(flags.item()) & 1


def test_conv2d_x6_flags_overflow(gpu):
    """The direct 3x3 kernel raises DD_NUM_F16_OVERFLOW_BIT too."""
    x = rnd(1, 32, 16, 16, seed=15)
    x[0, 5, 7, 9] = 1e6
    w = rnd(64, 32, 3, 3, seed=16)
    out = torch.empty(1, 16, 16, 64, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1))
    ok(gpu.dd_op_conv2d_x3(xin.data_ptr(), 1, 16, 16, 32, win.data_ptr(), None, None, out.data_ptr(), 64, 3, 3, 1,
                           1, 0, 0, flags.data_ptr(), None), gpu)
    assert int(flags.item()) & 1


@pytest.mark.parametrize("M,K,N,relu", [(1, 256, 1024, False), (1280, 256, 256, True), (4096, 320, 256, True),
                                        (600, 1024, 24, False), (77, 8, 256, False), (1280, 256, 1, False),
                                        (20, 512, 768, True), (4096, 512, 64, False), (4160, 256, 512, True)])
def test_gemm(gpu, M, K, N, relu):
    a = rnd(M, K, seed=5)
    w = rnd(N, K, seed=6, scale=1.0 / np.sqrt(K))
    b = rnd(N, seed=7)
    r = rnd(M, N, seed=8)
    ref = a @ w.T + b + r
    if relu:
        ref = F.relu(ref)
    out = torch.empty(M, N, device=DEV)
    ad, wd, bd, rd = g(a), g(w), g(b), g(r)
    ok(gpu.dd_op_gemm(ad.data_ptr(), M, K, wd.data_ptr(), bd.data_ptr(), rd.data_ptr(), out.data_ptr(), N,
                      int(relu), None), gpu)
    close(out, ref, 2e-5)


@pytest.mark.parametrize("batch,M,N,K,kn", [(8, 320, 320, 16, 0), (8, 320, 16, 320, 1), (4, 320, 128, 320, 1),
                                             (3, 70, 50, 36, 0)])
def test_gemm_batched(gpu, batch, M, N, K, kn):
    a = rnd(batch, M, K, seed=9)
    bm = rnd(batch, K, N, seed=10) if kn else rnd(batch, N, K, seed=10)
    ref = a @ (bm if kn else bm.transpose(1, 2))
    out = torch.empty(batch, M, N, device=DEV)
    ad, bd = g(a), g(bm)
    ok(gpu.dd_op_gemm_batched(ad.data_ptr(), bd.data_ptr(), out.data_ptr(), batch, M, N, K, kn, None), gpu)
    close(out, ref, 2e-5)


@pytest.mark.parametrize("rows,C,res_div,film", [(1000, 256, 0, False), (333, 64, 20, True), (50, 2048, 0, False),
                                                 (20, 1024, 4, False), (77, 128, 0, True), (129, 512, 3, False),
                                                 (45, 320, 0, False)])
def test_layernorm(gpu, rows, C, res_div, film):
    x = rnd(rows, C, seed=11, scale=3.0) + 0.5
    gam, bet = rnd(C, seed=12), rnd(C, seed=13)
    res = rnd((rows + res_div - 1) // res_div if res_div else rows, C, seed=14) if res_div else None
    fs, fb = (rnd(C, seed=15), rnd(C, seed=16)) if film else (None, None)
    xin = x + (res.repeat_interleave(res_div, 0)[:rows] if res_div else 0)
    ref = F.layer_norm(xin, (C,), gam, bet, 1e-5)
    if film:
        ref = ref * (1 + fs) + fb
    out = torch.empty(rows, C, device=DEV)
    keep = [g(t) if t is not None else None for t in (x, res, gam, bet, fs, fb)]
    p = [t.data_ptr() if t is not None else None for t in keep]
    ok(gpu.dd_op_layernorm(p[0], p[1], max(res_div, 1), p[2], p[3], p[4], p[5], out.data_ptr(), rows, C, None), gpu)
    close(out, ref, 1e-5)


def test_softmax(gpu):
    x = rnd(777, 320, seed=17, scale=4.0)
    ref = torch.softmax(x * 0.125, -1)
    xg = g(x)
    ok(gpu.dd_op_softmax_rows(xg.data_ptr(), 777, 320, 0.125, None), gpu)
    close(xg, ref, 1e-6)


@pytest.mark.parametrize("B,Hi,Wi,C,Ho,Wo", [(2, 8, 32, 64, 64, 256), (2, 8, 8, 256, 64, 64), (1, 16, 16, 64, 64, 64),
                                             (2, 64, 64, 7, 128, 256), (1, 8, 8, 12, 16, 16)])
def test_bilinear(gpu, B, Hi, Wi, C, Ho, Wo):
    x = rnd(B, C, Hi, Wi, seed=18)
    ref = F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=False)
    out = torch.empty(B, Ho, Wo, C, device=DEV)
    xd = g(x.permute(0, 2, 3, 1))
    ok(gpu.dd_op_bilinear(xd.data_ptr(), B, Hi, Wi, C, out.data_ptr(), Ho, Wo, None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 1e-6)


@pytest.mark.parametrize("B,Hi,Wi,C,Ho,Wo", [(2, 8, 32, 64, 64, 256), (3, 8, 8, 128, 32, 32), (2, 8, 32, 512, 8, 32),
                                             (1, 8, 8, 12, 16, 16), (1, 8, 32, 36, 13, 50)])
def test_bilinear_add(gpu, B, Hi, Wi, C, Ho, Wo):
    """The trunk upsample-add (wide-issue bilinear_add4_kernel for float4 channels, the scalar form otherwise):
    bit-identical to base + F.interpolate's fp32 value computed in the same order."""
    x = rnd(B, C, Hi, Wi, seed=28)
    base = rnd(B, C, Ho, Wo, seed=29)
    ref = base + F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=False)
    out = g(base.permute(0, 2, 3, 1))
    xd = g(x.permute(0, 2, 3, 1))
    ok(gpu.dd_op_bilinear_add(xd.data_ptr(), B, Hi, Wi, C, out.data_ptr(), Ho, Wo, None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 1e-6)


def test_maxpool(gpu):
    x = rnd(2, 64, 37, 50, seed=19)
    ref = F.max_pool2d(x, 3, 2, 1)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    xd = g(x.permute(0, 2, 3, 1))
    ok(gpu.dd_op_maxpool3x3s2(xd.data_ptr(), 2, 37, 50, 64, out.data_ptr(), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 0.0)


@pytest.mark.parametrize("H,W,oh,ow", [(64, 256, 8, 32), (16, 16, 8, 8), (8, 32, 8, 32)])
def test_avgpool(gpu, H, W, oh, ow):
    x = rnd(2, 64, H, W, seed=20)
    ref = F.adaptive_avg_pool2d(x, (oh, ow))
    out = torch.empty(2, oh, ow, 64, device=DEV)
    xd = g(x.permute(0, 2, 3, 1))
    ok(gpu.dd_op_avgpool(xd.data_ptr(), 2, H, W, 64, oh, ow, out.data_ptr(), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 1e-6)


def test_bev_sample_attn(gpu):
    B, Q, P, H, W, C = 3, 20, 8, 64, 64, 256
    logits = rnd(B, Q, P, seed=21, scale=2.0)
    pts = rnd(B, Q, P, 2, seed=22, scale=20.0)
    pts[0, 0, 0] = torch.tensor([40.0, -50.0])  # outside the BEV: zero padding
    pts[0, 0, 1] = torch.tensor([31.7, 31.9])   # partially outside
    value = rnd(B, C, H, W, seed=23)
    grid = torch.stack([pts[..., 1] / 32.0, pts[..., 0] / 32.0], -1)
    s = F.grid_sample(value, grid, mode="bilinear", padding_mode="zeros", align_corners=False)
    ref = (torch.softmax(logits, -1).unsqueeze(1) * s).sum(-1).permute(0, 2, 1)
    out = torch.empty(B, Q, C, device=DEV)
    ld, pd, vd = g(logits), g(pts), g(value.permute(0, 2, 3, 1))
    ok(gpu.dd_op_bev_sample_attn(ld.data_ptr(), pd.data_ptr(), vd.data_ptr(), out.data_ptr(), B, Q, P, H, W, C,
                                 None), gpu)
    close(out, ref, 1e-5)


@pytest.mark.parametrize("Lq,Lk", [(31, 31), (31, 65), (20, 30), (20, 1), (5, 128)])
def test_mha_small(gpu, Lq, Lk):
    B, nh, hd = 3, 8, 32
    q, k, v = rnd(B, Lq, nh * hd, seed=24), rnd(B, Lk, nh * hd, seed=25), rnd(B, Lk, nh * hd, seed=26)
    qh = q.view(B, Lq, nh, hd).transpose(1, 2)
    kh = k.view(B, Lk, nh, hd).transpose(1, 2)
    vh = v.view(B, Lk, nh, hd).transpose(1, 2)
    ref = (torch.softmax(qh @ kh.transpose(-1, -2) / np.sqrt(hd), -1) @ vh).transpose(1, 2).reshape(B, Lq, nh * hd)
    out = torch.empty(B, Lq, nh * hd, device=DEV)
    qd, kd, vd = g(q), g(k), g(v)
    ok(gpu.dd_op_mha_small(qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), B, Lq, Lk, nh, hd, None), gpu)
    close(out, ref, 1e-5)


@pytest.mark.parametrize("B,T,C", [(2, 320, 64), (2, 320, 128), (1, 320, 256), (1, 320, 512), (1, 64, 1024),
                                   (1, 320, 2048), (1, 128, 256)])
def test_gpt_attention(gpu, B, T, C):
    """Fused GPT self-attention (transfuser_backbone.py:386-410), fp32-MFMA form, vs the PyTorch fp32
    restatement."""
    nh, hs = 4, C // 4
    qkv = rnd(B, T, 3 * C, seed=31)
    q, k, v = (t.reshape(B, T, nh, hs).transpose(1, 2) for t in qkv.split(C, -1))
    att = torch.softmax((q @ k.transpose(-2, -1)) * (1.0 / np.sqrt(hs)), -1)
    ref = (att @ v).transpose(1, 2).reshape(B, T, C)
    out = torch.empty(B, T, C, device=DEV)
    qd = g(qkv)
    ok(gpu.dd_op_gpt_attention(qd.data_ptr(), out.data_ptr(), B, T, C, nh, 0, None), gpu)
    close(out, ref, 2e-5)


@pytest.mark.parametrize("B,T,C,amp", [(2, 320, 64, 1.0), (2, 320, 128, 1.0), (1, 320, 256, 1.0), (1, 320, 512, 1.0),
                                       (1, 320, 512, 4.0), (2, 64, 128, 1.0), (1, 96, 64, 3.0),
                                       # T / 32 = 8, 16, 24: wave counts 4 / 4 / 4 (not the 10 of T = 320)
                                       (1, 256, 256, 1.0), (1, 512, 128, 1.0), (1, 768, 64, 1.0), (1, 224, 512, 1.0)])
@pytest.mark.parametrize("prec", [1, 2])
def test_gpt_attention_f16x3(gpu, B, T, C, amp, prec):
    """The f16x3 GPT attention (flash-style over 32-key tiles, P taken from the S^T accumulators) vs PyTorch
    fp64; amp scales q / k to sharpen the softmax (scores up to ~|40| at amp 4). prec 1: scores on two-way
    splits (three products), prec 2: three-way splits (six products) - the same fp32-class bar."""
    nh, hs = 4, C // 4
    qkv = rnd(B, T, 3 * C, seed=33)
    qkv[..., : 2 * C] *= amp
    q, k, v = (t.double().reshape(B, T, nh, hs).transpose(1, 2) for t in qkv.split(C, -1))
    att = torch.softmax((q @ k.transpose(-2, -1)) * (1.0 / np.sqrt(hs)), -1)
    ref = (att @ v).transpose(1, 2).reshape(B, T, C)
    out = torch.empty(B, T, C, device=DEV)
    qd = g(qkv)
    ok(gpu.dd_op_gpt_attention(qd.data_ptr(), out.data_ptr(), B, T, C, nh, prec, None), gpu)
    close(out, ref, 2e-5)


@pytest.mark.parametrize("B,H,W", [(2, 64, 256), (1, 256, 256), (1, 40, 72), (2, 37, 50)])
def test_stem_pool_f16x3(gpu, B, H, W):
    """Fused stem conv 7x7/2 + bias + ReLU + maxpool 3x3/2 (transfuser_backbone.py:23-33) vs PyTorch fp64."""
    x = rnd(B, 4, H, W, seed=41).abs()
    x[:, 3] = 0.0  # the padded 4th input channel
    w = rnd(64, 4, 7, 7, seed=42, scale=1.0 / np.sqrt(196))
    b = rnd(64, seed=43)
    ref = F.max_pool2d(F.relu(F.conv2d(x.double(), w.double(), b.double(), 2, 3)), 3, 2, 1)
    out = torch.empty(ref.permute(0, 2, 3, 1).shape, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    xin, win, bin_ = g(x.permute(0, 2, 3, 1)), g(w.permute(0, 2, 3, 1)), g(b)
    ok(gpu.dd_op_stem_pool_x3(xin.data_ptr(), B, H, W, win.data_ptr(), bin_.data_ptr(), out.data_ptr(),
                              flags.data_ptr(), None), gpu)
    close(out.permute(0, 3, 1, 2), ref, 3e-5)
    assert int(flags.item()) == 0


@pytest.mark.parametrize("K,N", [(256, 256), (512, 256), (256, 1024), (1024, 256)])
def test_mk_linear_core(gpu, K, N):
    """The decoder megakernel's GEMM core (LDS split + fragment-order f16x3 weights + 32x32x16 MFMA) vs
    PyTorch fp64: 32 rows, fp32-class tolerance."""
    a = rnd(32, K, seed=91)
    w = rnd(N, K, seed=92, scale=1.0 / np.sqrt(K))
    b = rnd(N, seed=93)
    ref = a.double() @ w.double().T + b.double()
    out = torch.empty(32, N, device=DEV)
    ad, wd, bd = g(a), g(w), g(b)
    ok(gpu.dd_op_mk_linear(ad.data_ptr(), K, wd.data_ptr(), bd.data_ptr(), out.data_ptr(), N, None), gpu)
    close(out, ref, 3e-5)


@pytest.mark.parametrize("B", [1, 3])
def test_bevproj_fused(gpu, B):
    """bevproj.hip: LayerNorm(ReLU(bilinear(kvp 8x8 -> 64x64) + p3 W_p3^T + b)) in one pass vs PyTorch fp64
    on the same decomposition (transfuser_model_v2.py:123-140 with the keyval half projected at 8 x 8);
    p3 strided inside a 320-channel concat buffer as in the forward."""
    H = W = 64
    cat = rnd(B * H * W, 320, seed=101)
    p3 = cat[:, 256:]
    kvp = rnd(B, 8, 8, 256, seed=102)
    w = rnd(256, 64, seed=103, scale=1.0 / 8.0)
    bias = rnd(256, seed=104)
    lg, lb = 1.0 + 0.1 * rnd(256, seed=105), rnd(256, seed=106)
    bil = F.interpolate(kvp.double().permute(0, 3, 1, 2), size=(H, W), mode="bilinear", align_corners=False)
    v = F.relu(p3.double() @ w.double().T + bias.double() + bil.permute(0, 2, 3, 1).reshape(-1, 256))
    ref = F.layer_norm(v, (256,), lg.double(), lb.double(), 1e-5)
    out = torch.empty(B * H * W, 256, device=DEV)
    cd, kd, wd, bd, gd, ld = g(cat), g(kvp), g(w), g(bias), g(lg), g(lb)
    ok(gpu.dd_op_bevproj(cd.data_ptr() + 256 * 4, 320, kd.data_ptr(), wd.data_ptr(), bd.data_ptr(), gd.data_ptr(),
                         ld.data_ptr(), out.data_ptr(), B, H, W, 8, 8, None), gpu)
    close(out, ref, 3e-5)
