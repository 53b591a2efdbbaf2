"""End-to-end parity of the MI355X forward (through the C ABI) against the reference goldens.

Goldens: ``tests/golden/ref_b{B}_s{seed}.npz`` were produced by running the REFERENCE model
(``/root/reference``, shimmed imports) on seeded weights/inputs (``tests/golden/make_golden.py``).
Bar (BASELINE.json north star): per-scene waypoint L2 <= 1e-4 (max over the batch), written
here as ``WAYPOINT_L2_TOL``; headings and every per-(step, layer) decoder output are checked with
the same absolute bound; intermediates are checked on strided samples + checksums.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import compare_tap, golden_files, golden_files_r50, load, waypoint_l2

pytestmark = pytest.mark.gpu

WAYPOINT_L2_TOL = 1e-4
HEADING_TOL = 1e-4
MODE_TOL = 1e-4    # absolute, on every per-(step, layer) poses_reg (m / rad) and poses_cls (logit)
# absolute, agent_states (m / rad) and labels. The agent head (x, y = tanh * 32) is ill-conditioned on the
# seeded weights: the REFERENCE's own agent_states move by 1.6e-4 when the camera input is perturbed by one
# fp32 ulp (2^-24 relative; tests/test_conditioning.py measures it), and the fp32-MFMA path sits at 2.5e-4 from
# the goldens by summation order alone. f16x3 carries ~4-8x fp32's rounding per contraction, so the bar is 10x
# the one-ulp response (test_conditioning asserts that relation stays true).
AGENT_TOL = 2e-3
TAP_TOL = 2e-5  # relative to max(1, |sample|max) on intermediates


def _nchw(t, B, H, W, C):
    return t[: B * H * W * C].view(B, H, W, C).permute(0, 3, 1, 2).contiguous()


def _report(lines):
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "parity_report.txt"), "a") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


GEMM_MODES = ["fp32", "f16x3"]


@pytest.mark.parametrize("mode", GEMM_MODES)
@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_forward_matches_reference_goldens(gpu_model, path, mode):
    _check_golden(gpu_model, path, mode)


def _check_golden(model, path, mode, cfg=None):
    """Run the golden's batch through ``model`` in ``mode`` and hold the trajectory, every per-(step, layer)
    poses_reg / poses_cls, the agent outputs and the intermediates to the bars above."""
    from diffusiondrive_amd.weights import synthetic_inputs
    model.set_gemm_mode(mode)
    g = load(path)
    B, seed = int(g["batch"]), int(g["seed"])
    inp = synthetic_inputs(B, seed, cfg)
    assert np.array_equal(inp["noise"], g["noise"])
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    out = model.forward(feats, noise=torch.from_numpy(inp["noise"]), heads=True, modes=True)
    lines = [f"== {os.path.basename(path)} B={B} gemm={mode}"]
    l2 = waypoint_l2(out["trajectory"].numpy(), g["trajectory"])
    hd = float(np.abs(out["trajectory"].numpy()[..., 2] - g["trajectory"][..., 2]).max())
    lines.append(f"trajectory: waypoint L2 max {l2:.3e}  heading max {hd:.3e}")
    errs = {}
    for s in range(2):
        for l in range(2):
            reg = model.tap(f"reg_s{s}l{l}", (B, 20, 8, 3)).cpu().numpy()
            cls = model.tap(f"cls_s{s}l{l}", (B, 20)).cpu().numpy()
            errs[f"reg_s{s}l{l}"] = float(np.abs(reg - g[f"reg_s{s}l{l}"]).max())
            errs[f"cls_s{s}l{l}"] = float(np.abs(cls - g[f"cls_s{s}l{l}"]).max())
    errs["agent_states"] = float(np.abs(out["agent_states"].numpy() - g["agent_states"]).max())
    errs["agent_labels"] = float(np.abs(out["agent_labels"].numpy() - g["agent_labels"]).max())
    c4 = int(g["tap_img_l4_shape"][1])   # 512 (ResNet-34) / 2048 (ResNet-50)
    taps = {
        "img_l4": _nchw(model.tap("img_l4"), B, 8, 32, c4),
        "p3": _nchw(model.tap("cross_in"), B, 64, 64, 320)[:, 256:],
        "bev_feature": _nchw(model.tap("bev_feature"), B, 8, 8, 512),
        "keyval": model.tap("keyval", (B, 65, 256)),
        "cross_bev_tokens": model.tap("cross_bev", (B, 4096, 256)),
        "query_out": model.tap("query_out", (B, 31, 256)),
        "bev_semantic_map": out["bev_semantic_map"],
    }
    for s in range(2):
        for l in range(2):
            taps[f"gs_s{s}l{l}"] = model.tap(f"gs_s{s}l{l}", (B, 20, 256))
    if mode != "f16x3":  # f16x3 evaluates value_proj only at the sampled taps (test below)
        for l in range(2):
            taps[f"value_call{l}_l{l}"] = _nchw(model.tap(f"value_l{l}"), B, 64, 64, 256)
    tap_errs = {k: compare_tap(g, k, v.cpu().numpy()) for k, v in taps.items()}
    for k, v in errs.items():
        lines.append(f"  {k:22s} max abs err {v:.3e}")
    for k, (e, cs) in tap_errs.items():
        lines.append(f"  tap {k:18s} sample rel err {e:.3e}  checksum rel err {cs:.3e}")
    _report(lines)
    assert model.numerics_flags() == 0
    assert l2 <= WAYPOINT_L2_TOL, f"waypoint L2 {l2:.3e} > {WAYPOINT_L2_TOL}"
    assert hd <= HEADING_TOL
    for k, v in errs.items():
        assert v <= (AGENT_TOL if k.startswith("agent") else MODE_TOL), (k, v)
    for k, (e, cs) in tap_errs.items():
        assert e <= TAP_TOL and cs <= TAP_TOL, (k, e, cs)


@pytest.mark.parametrize("mode", GEMM_MODES)
def test_forward_graph_replay_is_deterministic(gpu_model, mode):
    """Second and third calls replay the captured hipGraph: results must be bit-identical."""
    from diffusiondrive_amd.weights import synthetic_inputs
    gpu_model.set_gemm_mode(mode)
    inp = synthetic_inputs(2, 99)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    a = gpu_model.forward(feats, noise=nz)["trajectory"]
    b = gpu_model.forward(feats, noise=nz)["trajectory"]
    c = gpu_model.forward(feats, noise=nz)["trajectory"]
    assert torch.equal(a, b) and torch.equal(b, c)


@pytest.mark.parametrize("mode", GEMM_MODES)
def test_forward_matches_oracle_batch8(gpu_model, seeded_sd, mode):
    """Wider check vs the golden-pinned CPU oracle on an unseen seed (B=8)."""
    from oracle.model import OracleModel
    gpu_model.set_gemm_mode(mode)
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(8, 4321)
    ref = OracleModel(seeded_sd).forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"],
                                         inp["noise"], heads=False)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    out = gpu_model.forward(feats, noise=torch.from_numpy(inp["noise"]), modes=True)
    l2 = waypoint_l2(out["trajectory"].numpy(), ref["trajectory"].numpy())
    _report([f"== oracle B=8 seed 4321 gemm={mode}: waypoint L2 {l2:.3e}, "
             f"modes max err {float((out['poses_reg'] - ref['poses_reg']).abs().max()):.3e}"])
    assert gpu_model.numerics_flags() == 0
    assert l2 <= WAYPOINT_L2_TOL


@pytest.fixture(scope="module")
def r50_model(gpu):
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import seeded_state_dict
    cfg = TransfuserConfig(image_architecture="resnet50")
    return DiffusionDriveModel(cfg, seeded_state_dict(cfg, 3), device=0), cfg


@pytest.mark.parametrize("mode", GEMM_MODES)
@pytest.mark.parametrize("path", golden_files_r50(), ids=os.path.basename)
def test_resnet50_config_matches_oracle(r50_model, path, mode):
    """BASELINE config C4: ResNet-50 image trunk (TransfuserConfig.image_architecture="resnet50",
    transfuser_config.py:17; LiDAR stays ResNet-34, channels adapt via transfuser_backbone.py:66-93) against
    the REFERENCE's own C4 goldens (make_golden.py ``B:seed:r50``, B = 2 and 4; the oracle is pinned to the
    same files in test_oracle_golden.py): trajectory, every per-(step, layer) reg / cls, the Bottleneck
    trunk's layer-4 output and the downstream taps at the bars of the ResNet-34 goldens."""
    m, cfg = r50_model
    _check_golden(m, path, mode, cfg)


@pytest.mark.parametrize("mode", GEMM_MODES)
def test_vanilla_ddim_schedule_matches_oracle(gpu_model, seeded_sd, mode):
    """C5 ablation: 10-step vanilla (non-truncated) DDIM on the same decoder vs the oracle's
    restatement of diffusers' leading set_timesteps(10) (no reference counterpart)."""
    from oracle.model import OracleModel
    from diffusiondrive_amd.weights import synthetic_inputs
    gpu_model.set_gemm_mode(mode)
    inp = synthetic_inputs(2, 555)
    ref = OracleModel(seeded_sd).forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"],
                                         inp["noise"], steps=10, heads=False, schedule="vanilla")
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    gpu_model.set_schedule("vanilla")
    try:
        out = gpu_model.forward(feats, noise=torch.from_numpy(inp["noise"]), steps=10)
    finally:
        gpu_model.set_schedule("truncated")
    l2 = waypoint_l2(out["trajectory"].numpy(), ref["trajectory"].numpy())
    _report([f"== vanilla DDIM 10 steps B=2 gemm={mode}: waypoint L2 vs oracle {l2:.3e}"])
    assert l2 <= WAYPOINT_L2_TOL


# bf16 mode (configs C2-bf16 / C4: one bf16 product per MAC in the backbone, f16x3 after it) is NOT a parity
# mode: a near-tie of the 20 cls logits can flip the selected mode. Its bar is on the PRE-argmax tensors against
# the fp32 oracle: every mode's 8 waypoints (last step, last layer; per-mode L2, max over scenes and modes), every
# cls logit and the mode agreement (argmax equal) must be no worse than BOTH a fixed bar (SURVEY §8a's measured
# bf16-autocast class: 0.06-0.08 m) AND the reference path's own bf16 (the oracle under torch.autocast(cpu,
# bfloat16)) on the same batch - each statistic is held to the stricter of the two.
BF16_ALLMODE_TOL = 0.1   # m
BF16_CLS_TOL = 0.1       # logit
BF16_AGREE = 0.9


def _bf16_stats(out, ref, B):
    reg, rreg = out["poses_reg"].float().numpy(), ref["poses_reg"].numpy()
    return {"allmode": waypoint_l2(reg.reshape(B * 20, 8, 3), rreg.reshape(B * 20, 8, 3)),
            "cls": float(np.abs(out["poses_cls"].float().numpy() - ref["poses_cls"].numpy()).max()),
            "agree": float((out["poses_cls"].float().numpy().argmax(-1) == ref["poses_cls"].numpy().argmax(-1)).mean()),
            "sel": waypoint_l2(out["trajectory"].float().numpy(), ref["trajectory"].numpy())}


def _bf16_bar(out, om, args, B, tag):
    ref = om.forward(*args, heads=False)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ac = _bf16_stats(om.forward(*args, heads=False), ref, B)
    st = _bf16_stats(out, ref, B)
    _report([f"== {tag}: all-mode waypoint L2 {st['allmode']:.3e} m (reference bf16 autocast {ac['allmode']:.3e}), "
             f"cls max dev {st['cls']:.3e} ({ac['cls']:.3e}), mode agreement {st['agree']:.3f} ({ac['agree']:.3f}), "
             f"selected-trajectory L2 {st['sel']:.3e} ({ac['sel']:.3e}) [bf16: reduced precision]"])
    assert st["allmode"] <= min(BF16_ALLMODE_TOL, ac["allmode"]), (st, ac)
    assert st["cls"] <= min(BF16_CLS_TOL, ac["cls"]), (st, ac)
    assert st["agree"] >= max(BF16_AGREE, ac["agree"]), (st, ac)


def test_bf16_mode_resnet34(gpu_model, seeded_sd):
    """C2-bf16: ResNet-34, B = 8, vs the fp32 oracle under the bf16 bar."""
    from oracle.model import OracleModel
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(8, 1234)
    args = (inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"])
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    gpu_model.set_gemm_mode("bf16")
    try:
        out = gpu_model.forward(feats, noise=torch.from_numpy(inp["noise"]), modes=True)
    finally:
        gpu_model.set_gemm_mode("fp32")
    _bf16_bar(out, OracleModel(seeded_sd), args, 8, "bf16 resnet34 B=8")


def test_bf16_resnet50_batch64_config_c4():
    """BASELINE config C4 as stated: ResNet-50 image trunk (transfuser_backbone.py:67-93 channel adaptation),
    bf16, B = 64, vs the fp32 CPU oracle under the bf16 bar (every conv of the trunks on the bf16 conv_x6 /
    stem_pool / conv_x3 kernels)."""
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
    from oracle.model import OracleModel
    cfg = TransfuserConfig(image_architecture="resnet50")
    sd = seeded_state_dict(cfg, 3)
    B = 64
    inp = synthetic_inputs(B, 1234, cfg)
    args = (inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"])
    m = DiffusionDriveModel(cfg, sd, device=0, gemm="bf16")
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    out = m.forward(feats, noise=torch.from_numpy(inp["noise"]), modes=True)
    assert m.numerics_flags() == 0
    # the scenes are independent (eval-mode BN, per-scene decoder), so the CPU oracle checks the first and the last
    # eight of the 64 (the first and the last tiles of every batched kernel) - a quarter of its B = 64 cost
    sel = np.r_[0:8, B - 8:B]
    sub = {k: out[k][torch.from_numpy(sel)] for k in ("poses_reg", "poses_cls", "trajectory")}
    _bf16_bar(sub, OracleModel(sd, cfg), tuple(a[sel] for a in args), len(sel), "C4 resnet50 bf16 B=64 (16 scenes)")


def test_gathered_value_rows_match_dense_map(gpu_model):
    """f16x3 evaluates value_proj (blocks.py:68-76,114) only at the map pixels grid_sample's bilinear
    taps read (blocks.py:101-122), each distinct pixel of a scene once (conv_x3 gathered rows, the scenes'
    rows compacted into full tiles by their counts):
    the tap geometry must follow align_corners=False / zero padding, each scene's row list must be
    exactly its distinct tap pixels in pixel order (-1 past the count), every tap's slot must hold
    its pixel (-1 for zero-padded taps), and every gathered row must equal the fp32 dense map at its
    pixel. Checked on step 1 / layer 0, whose points are the ``pts`` buffer at the end of the
    forward; the dense map does not depend on the points."""
    from diffusiondrive_amd.weights import synthetic_inputs
    B, Q, P, HB = 4, 20, 8, 64
    cap = Q * P * 4
    inp = synthetic_inputs(B, 5)
    # push some points off the 64 x 64 BEV map so zero-padded taps are exercised
    nz = inp["noise"].copy()
    nz[:, :3] *= 40.0
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    gpu_model.set_gemm_mode("fp32")
    gpu_model.forward(feats, noise=torch.from_numpy(nz))
    dense = gpu_model.tap("value_l0", (B, HB, HB, 256)).double().cpu().numpy().reshape(-1, 256)
    gpu_model.set_gemm_mode("f16x3")
    try:
        gpu_model.forward(feats, noise=torch.from_numpy(nz))
        n = B * cap
        rows = gpu_model.tap("value_taps_s1l0")[:n].view(torch.int32).cpu().numpy()
        slots = gpu_model.tap("value_slots_s1l0")[:n].view(torch.int32).cpu().numpy()
        counts = gpu_model.tap("value_cnt_s1l0")[:B].view(torch.int32).cpu().numpy()
        vals = gpu_model.tap("value_rows_s1l0", (n, 256)).double().cpu().numpy()
        pts = gpu_model.tap("pts", (B * Q * P, 2)).double().cpu().numpy()
    finally:
        gpu_model.set_gemm_mode("fp32")
    # tap geometry (float32 arithmetic as the kernel / F.grid_sample)
    p32 = pts.astype(np.float32)
    ix = ((p32[:, 1] / np.float32(32) + 1) * np.float32(HB) - 1) / 2
    iy = ((p32[:, 0] / np.float32(32) + 1) * np.float32(HB) - 1) / 2
    x0, y0 = np.floor(ix).astype(np.int64), np.floor(iy).astype(np.int64)
    b = np.arange(B * Q * P) // (Q * P)
    pix = []
    for dy, dx in ((0, 0), (0, 1), (1, 0), (1, 1)):
        yy, xx = y0 + dy, x0 + dx
        ok = (yy >= 0) & (yy < HB) & (xx >= 0) & (xx < HB)
        pix.append(np.where(ok, (b * HB + yy) * HB + xx, -1))
    pix = np.stack(pix, 1).reshape(-1)
    assert (pix < 0).any() and (pix >= 0).any()
    for s_ in range(B):
        tp = pix[s_ * cap:(s_ + 1) * cap]
        uniq = np.unique(tp[tp >= 0])
        rs = rows[s_ * cap:(s_ + 1) * cap]
        assert np.array_equal(rs[:len(uniq)], uniq) and (rs[len(uniq):] == -1).all(), s_
        assert counts[s_] == len(uniq), (s_, counts[s_], len(uniq))  # the compacted launch's row counts
    assert np.array_equal(slots < 0, pix < 0)
    live = slots >= 0
    assert np.array_equal(rows[slots[live]], pix[live])
    used = rows >= 0
    ref = dense[rows[used]]
    err = np.abs(vals[used] - ref).max() / max(1.0, np.abs(ref).max())
    assert err <= TAP_TOL, err


def test_decoder_megakernel_matches_unfused_chain(gpu_model, seeded_sd, monkeypatch):
    """The f16x3 trajectory head runs as the decoder megakernel (decoder_mk.hip: 1 + 2 launches per
    (step, layer) counting the gathered value_proj conv); DDMI_DECODER_MK=0 keeps the unfused per-op chain.
    Both on the same inputs: every per-(step, layer) poses_reg / poses_cls and the BEV-attention aggregate
    within the 1e-4 bar, and the megakernel proven dispatched (launch count of the "decoder" class)."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 4
    inp = synthetic_inputs(B, 31)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    gpu_model.set_gemm_mode("f16x3")
    try:
        gpu_model.set_profiling(True)
        gpu_model.reset_stats()
        out = gpu_model.forward(feats, noise=nz)["trajectory"].numpy()
        st = gpu_model.kernel_stats("decoder")
        gpu_model.set_profiling(False)
        got = {f"{k}_s{s}l{l}": gpu_model.tap(f"{k}_s{s}l{l}").cpu().numpy()[: B * 20 * (24 if k == "reg" else
                                                                                    256 if k == "gs" else 1)]
               for k in ("reg", "cls", "gs") for s in range(2) for l in range(2)}
    finally:
        gpu_model.set_profiling(False)
        gpu_model.set_gemm_mode("fp32")
    assert st["launches"] == 1 + 2 * 2, st  # init + one per (step, layer)
    monkeypatch.setenv("DDMI_DECODER_MK", "0")
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    m.set_profiling(True)
    ref_out = m.forward(feats, noise=nz)["trajectory"].numpy()
    assert m.kernel_stats("decoder")["launches"] == 0
    m.set_profiling(False)
    lines = ["== decoder megakernel vs unfused chain (f16x3, B=4)"]
    for k, v in got.items():
        r = m.tap(k).cpu().numpy()[: v.size]
        err = float(np.abs(v - r).max())
        lines.append(f"  {k:10s} max abs err {err:.3e}")
        assert err <= MODE_TOL * (1 if not k.startswith("gs") else max(1.0, np.abs(r).max())), (k, err)
    l2 = waypoint_l2(out, ref_out)
    lines.append(f"  trajectory waypoint L2 {l2:.3e}")
    _report(lines)
    assert l2 <= WAYPOINT_L2_TOL


def test_tf_decoder_megakernel_matches_unfused_chain(gpu_model, seeded_sd, monkeypatch):
    """The f16x3 _tf_decoder (3 post-norm layers) plus the trajectory head's agent K / V and ego-attention
    hoists run as ONE megakernel launch (tfdec_mk.hip); DDMI_TFDEC_MK=0 keeps the unfused chain. Same
    inputs: the decoded queries, the hoisted agent K / V and ego rows within the 1e-4 bar (relative to the
    tensor's scale), the trajectory within the waypoint bar, and the megakernel proven dispatched."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 4
    inp = synthetic_inputs(B, 37)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    sizes = {"query_out": B * 31 * 256, "agent_kv0": B * 30 * 512, "agent_kv1": B * 30 * 512, "ego_out0": B * 256,
             "ego_out1": B * 256}
    names = tuple(sizes)
    gpu_model.set_gemm_mode("f16x3")
    try:
        gpu_model.set_profiling(True)
        gpu_model.reset_stats()
        res = gpu_model.forward(feats, noise=nz)
        out = res["trajectory"].numpy()
        st = gpu_model.kernel_stats("tfdec")
        gpu_model.set_profiling(False)
        got = {k: gpu_model.tap(k).cpu().numpy()[: sizes[k]] for k in names}
    finally:
        gpu_model.set_profiling(False)
        gpu_model.set_gemm_mode("fp32")
    assert st["launches"] == 1, st
    monkeypatch.setenv("DDMI_TFDEC_MK", "0")
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    m.set_profiling(True)
    ref_out = m.forward(feats, noise=nz)["trajectory"].numpy()
    assert m.kernel_stats("tfdec")["launches"] == 0
    m.set_profiling(False)
    lines = ["== tf-decoder megakernel vs unfused chain (f16x3, B=4)"]
    for k, v in got.items():
        r = m.tap(k).cpu().numpy()[: sizes[k]]
        assert r.shape == v.shape, (k, r.shape, v.shape)
        err = float(np.abs(v - r).max())
        lines.append(f"  {k:10s} max abs err {err:.3e} (max |ref| {np.abs(r).max():.3e})")
        assert err <= MODE_TOL * max(1.0, float(np.abs(r).max())), (k, err)
    l2 = waypoint_l2(out, ref_out)
    lines.append(f"  trajectory waypoint L2 {l2:.3e}")
    _report(lines)
    assert l2 <= WAYPOINT_L2_TOL


@pytest.mark.parametrize("B", [1, 4, 16])
def test_tf_decoder_groups_match_one_workgroup(gpu_model, seeded_sd, monkeypatch, B):
    """The default tf-decoder megakernel runs four workgroups per scene (heads and FFN chunks split, three L2
    exchanges per layer, the linear2 K-slices summed in slab order); DDMI_TF_GROUPS=1 keeps one workgroup per
    scene with a single accumulation chain. Same products, linear2 re-associated: the decoded queries and hoists
    agree within the per-mode bar of the tensor's scale (measured 3e-6 relative at B = 1 / 4, 3.5e-5 at B = 16 - the
    largest of more rows; the megakernel and the unfused chain differ by as much), the trajectories within the
    waypoint bar, no numerics / sync-timeout flag is raised, and a second run of the four-workgroup kernel is
    bit-identical (the exchanges are race-free)."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(B, 43)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    sizes = {"query_out": B * 31 * 256, "agent_kv0": B * 30 * 512, "agent_kv1": B * 30 * 512, "ego_out0": B * 256,
             "ego_out1": B * 256}

    def run(m):
        m.set_gemm_mode("f16x3")
        try:
            m.numerics_flags(clear=True)
            out = m.forward(feats, noise=nz)["trajectory"].numpy()
            flags = m.numerics_flags(clear=True)
            taps = {k: m.tap(k).cpu().numpy()[: n] for k, n in sizes.items()}
        finally:
            m.set_gemm_mode("fp32")
        return out, taps, flags

    # the exchange buffers first hold another batch's values, so a stale read cannot pass as the right one
    other = synthetic_inputs(B, 44)
    gpu_model.set_gemm_mode("f16x3")
    try:
        gpu_model.forward({k: torch.from_numpy(other[k]) for k in feats}, noise=torch.from_numpy(other["noise"]))
    finally:
        gpu_model.set_gemm_mode("fp32")
    out4, taps4, f4 = run(gpu_model)
    out4b, taps4b, f4b = run(gpu_model)
    diff = {k: float(np.abs(taps4[k] - taps4b[k]).max()) for k in sizes if not np.array_equal(taps4[k], taps4b[k])}
    assert np.array_equal(out4, out4b) and not diff, (f4, f4b, float(np.abs(out4 - out4b).max()), diff)
    monkeypatch.setenv("DDMI_TF_GROUPS", "1")
    out1, taps1, f1 = run(DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3"))
    assert f4 == 0 and f1 == 0, (f4, f1)
    lines = [f"== tf-decoder megakernel, 4 workgroups per scene vs 1 (f16x3, B={B})"]
    for k in sizes:
        err = float(np.abs(taps4[k] - taps1[k]).max())
        lines.append(f"  {k:10s} max abs err {err:.3e} (max |ref| {np.abs(taps1[k]).max():.3e})")
        assert err <= MODE_TOL * max(1.0, float(np.abs(taps1[k]).max())), (k, err)
    l2 = waypoint_l2(out4, out1)
    lines.append(f"  trajectory waypoint L2 {l2:.3e}")
    _report(lines)
    assert l2 <= WAYPOINT_L2_TOL


def test_fused_token_pooling_matches_avgpool(gpu_model, seeded_sd, monkeypatch):
    """The GPT token pooling of every scale (adaptive avg-pool of the stage output to 8 x 32 / 8 x 8 tokens,
    + pos_emb; transfuser_backbone.py:241-276) runs inside the stage-final conv_x6 epilogue where conv_x6
    takes that conv; DDMI_FUSE_POOL=0 keeps the separate avgpool launches. Same arithmetic in the same
    order, so the forward is unchanged (1e-6); and the fused path is proven taken (fewer pool launches)."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 4
    inp = synthetic_inputs(B, 41)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    gpu_model.set_gemm_mode("f16x3")
    try:
        gpu_model.set_profiling(True)
        gpu_model.reset_stats()
        res = gpu_model.forward(feats, noise=nz)
        out = res["trajectory"].numpy()
        pools = gpu_model.kernel_stats("pool")["launches"]
        sizes = {"bev_feature": B * 64 * 512, "cross_in": B * 4096 * 320, "gpt_x": B * 320 * 512}
        taps = {k: gpu_model.tap(k).cpu().numpy()[:n] for k, n in sizes.items()}
    finally:
        gpu_model.set_profiling(False)
        gpu_model.set_gemm_mode("fp32")
    monkeypatch.setenv("DDMI_FUSE_POOL", "0")
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    m.set_profiling(True)
    ref = m.forward(feats, noise=nz)
    ref_pools = m.kernel_stats("pool")["launches"]
    m.set_profiling(False)
    assert ref_pools == 8, ref_pools  # 4 scales x (image, LiDAR)
    assert pools < ref_pools, (pools, ref_pools)
    for k, v in taps.items():
        assert float(np.abs(m.tap(k).cpu().numpy()[: v.size] - v).max()) <= 1e-6, k
    assert waypoint_l2(out, ref["trajectory"].numpy()) <= 1e-6


def test_value_proj_variants_agree(gpu_model, seeded_sd, monkeypatch):
    """The gathered value_proj on the same inputs: the default kernel (value_proj.hip: compacted rows in 256-row
    tiles, each tile as two 128-channel halves, the tile's 3 x 3-neighbourhood union staged once per 16-channel
    group, its K split over the channel groups 8 ways at this batch), the same tiles gathered per (row, tap)
    (DDMI_VPROJ_UNION=0), the union form with every tile / the larger-union tiles handed to the gathered fallback
    (DDMI_VPROJ_UMAX=0 / 600: bit-identical to the gathered form on those tiles), the union form unsplit and split 4
    ways (DDMI_VPROJ_USPLIT; the partials summed in split order by the last split), and conv_x3 over the compacted
    rows (DDMI_VALUE_SPLITK=0). The forms differ by summation order only: every live row within 1e-5 relative,
    trajectories within 1e-5."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 6
    inp = synthetic_inputs(B, 43)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    names = [f"s{s}l{l}" for s in range(2) for l in range(2)]

    def run(m, profile=False):
        if profile:
            m.set_profiling(True)
            m.reset_stats()
        out = m.forward(feats, noise=nz)["trajectory"].numpy()
        if profile:
            assert m.kernel_stats("value_proj")["launches"] == 4
            m.set_profiling(False)
        taps = {k: (m.tap(f"value_taps_{k}").view(torch.int32).cpu().numpy()[: B * 640],
                    m.tap(f"value_rows_{k}").cpu().numpy()[: B * 640 * 256].reshape(-1, 256)) for k in names}
        assert m.numerics_flags() == 0
        return out, taps

    def fresh(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
        try:
            return run(m)
        finally:
            m.close()
            for k in env:
                monkeypatch.delenv(k)

    gpu_model.set_gemm_mode("f16x3")
    try:
        runs = {"default": run(gpu_model, profile=True)}
    finally:
        gpu_model.set_profiling(False)
        gpu_model.set_gemm_mode("fp32")
    runs["gathered2"] = fresh(DDMI_VPROJ_UNION="0")
    runs["union_fb_all"] = fresh(DDMI_VPROJ_UMAX="0")
    runs["union_fb_some"] = fresh(DDMI_VPROJ_UMAX="600")
    runs["union_split1"] = fresh(DDMI_VPROJ_USPLIT="1")
    runs["union_split4"] = fresh(DDMI_VPROJ_USPLIT="4")
    runs["x3"] = fresh(DDMI_VALUE_SPLITK="0")
    ref_out, ref = runs["x3"]
    forms = ("default", "gathered2", "union_fb_some", "union_split1", "union_split4")
    lines = ["== gathered value_proj: value_proj.hip forms vs conv_x3 over the compacted rows"]
    for k in names:
        rows = ref[k][0]
        live = rows >= 0
        # every tile handed to the fallback: exactly the gathered two-half form
        assert np.array_equal(runs["union_fb_all"][1][k][1][live], runs["gathered2"][1][k][1][live]), k
        for v in forms:
            got = runs[v][1][k]
            assert np.array_equal(rows, got[0]), (v, k)
            r = ref[k][1][live]
            err = float(np.abs(got[1][live] - r).max() / max(1.0, np.abs(r).max()))
            lines.append(f"  {k} {v}: {int(live.sum())} live rows, max rel err vs conv_x3 {err:.3e}")
            assert err <= 1e-5, (v, k, err)
    assert np.array_equal(runs["union_fb_all"][0], runs["gathered2"][0])
    for v in forms:
        l2 = waypoint_l2(runs[v][0], ref_out)
        lines.append(f"  trajectory waypoint L2 {v} vs conv_x3 {l2:.3e}")
        assert l2 <= 1e-5, (v, l2)
    _report(lines)


@pytest.mark.parametrize("mode", ["f16x3", "bf16"])
def test_nchw_stem_equals_nhwc4_stem(gpu_model, seeded_sd, monkeypatch, mode):
    """The fused stems read the caller's NCHW camera / LiDAR tensors in place (through the handle's device input
    table) instead of an NHWC4 copy made by a transpose pass first (DDMI_STEM_NCHW=0): the same 4-channel pixels
    reach the same arithmetic, so the pooled stem maps and the trajectory are bit-identical - also on a forward
    whose inputs sit at new addresses (the captured graph reads the table, not a baked pointer)."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 3
    inp = synthetic_inputs(B, 47)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"]).cuda()
    gpu_model.set_gemm_mode(mode)
    try:
        a = gpu_model.forward(feats, noise=nz)["trajectory"].cpu().numpy()
        # replay (graph) with the same data at other device addresses
        moved = {k: v.clone() for k, v in feats.items()}
        b = gpu_model.forward(moved, noise=nz)["trajectory"].cpu().numpy()
        pools = [gpu_model.tap(n).cpu().numpy() for n in ("img_pool", "lid_pool")]
    finally:
        gpu_model.set_gemm_mode("fp32")
    monkeypatch.setenv("DDMI_STEM_NCHW", "0")
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm=mode)
    ref = m.forward(feats, noise=nz)["trajectory"].cpu().numpy()
    ref_pools = [m.tap(n).cpu().numpy() for n in ("img_pool", "lid_pool")]
    m.close()
    assert np.array_equal(a, ref) and np.array_equal(b, ref)
    for p, r in zip(pools, ref_pools):
        assert np.array_equal(p[: r.size], r[: p.size])


@pytest.mark.parametrize("mode", ["f16x3", "bf16"])
def test_gpt_layernorm_fold_is_bit_identical(gpu_model, seeded_sd, monkeypatch, mode):
    """The GPT blocks' LayerNorms at C <= 128 (ln2 after proj, ln1 of the next block / ln_f after the MLP-down) are
    written by the epilogue of the GEMM that produces their input (conv_x3's quad epilogue, one N tile per row,
    layernorm_v4's lane order and rounding): the LayerNorm outputs and therefore the whole forward are bit-identical
    to the separate launches (DDMI_LN_FOLD=0), and 8 LayerNorm launches per forward are gone."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 3
    inp = synthetic_inputs(B, 53)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"]).cuda()

    def run(m):
        m.set_profiling(True)
        m.reset_stats()
        out = m.forward(feats, noise=nz, modes=True)
        n_ln = m.kernel_stats("layernorm")["launches"]
        m.set_profiling(False)
        return {k: v.cpu().numpy() for k, v in out.items()}, n_ln, m.tap("gpt_h").cpu().numpy()

    gpu_model.set_gemm_mode(mode)
    try:
        fused, n_fused, h_fused = run(gpu_model)
    finally:
        gpu_model.set_gemm_mode("fp32")
    monkeypatch.setenv("DDMI_LN_FOLD", "0")
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm=mode)
    try:
        ref, n_ref, h_ref = run(m)
    finally:
        m.close()
    for k in ref:
        assert np.array_equal(fused[k], ref[k]), (mode, k)
    assert np.array_equal(h_fused[: h_ref.size], h_ref[: h_fused.size])  # ln_f of the last scale's tokens
    assert n_ref - n_fused == 8, (n_ref, n_fused)


@pytest.mark.parametrize("B", [3, 64])
def test_gpt_tail_fusion_is_bit_identical(gpu_model, seeded_sd, monkeypatch, B):
    """The C <= 128 GPT blocks' tail (proj + residual, ln2, MLP-up / ReLU / MLP-down + residual, the next LayerNorm)
    runs as one launch per block (gpt_tail.hip: the 4C hidden chunk by chunk in LDS) with the unfused chain's
    products, K order and epilogue expressions: the forward and the last scale's ln_f tokens are bit-identical to the
    proj / MLP-up / MLP-down launches (DDMI_GPT_TAIL=0), with 4 tail launches per forward in place of 12. The fused
    form is the default up to B = 16 and forced here (DDMI_GPT_TAIL=1) at B = 64 too."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(B, 57)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"]).cuda()

    def run(m):
        m.set_profiling(True)
        m.reset_stats()
        out = m.forward(feats, noise=nz, modes=True)
        n_tail = m.kernel_stats("gpt_tail")["launches"]
        m.set_profiling(False)
        return {k: v.cpu().numpy() for k, v in out.items()}, n_tail, m.tap("gpt_h").cpu().numpy()

    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DDMI_GPT_TAIL", flag)
        m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
        try:
            res[flag] = run(m)
        finally:
            m.close()
    (fused, n_fused, h_fused), (ref, n_ref, h_ref) = res["1"], res["0"]
    assert n_fused == 4 and n_ref == 0, (n_fused, n_ref)
    for k in ref:
        assert np.array_equal(fused[k], ref[k]), k
    assert np.array_equal(h_fused[: h_ref.size], h_ref[: h_fused.size])


@pytest.mark.parametrize("B", [16, 17])
def test_small_batch_forms_at_their_boundary(seeded_sd, B):
    """The small-batch forms switch by batch size (tf decoder four workgroups per scene and the fused GPT block tail
    up to B = 16, one workgroup / three launches above): at B = 16 and 17 the default handle's forward stays within
    the 1e-4 waypoint bar of the CPU oracle (the golden-pinned restatement) with no flag raised, and the profiler
    shows which forms ran."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    from oracle.model import OracleModel
    inp = synthetic_inputs(B, 71)
    ref = OracleModel(seeded_sd).forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"],
                                         inp["noise"], heads=False)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    try:
        m.set_profiling(True)
        m.reset_stats()
        out = m.forward(feats, noise=torch.from_numpy(inp["noise"]))
        n_tail = m.kernel_stats("gpt_tail")["launches"]
        m.set_profiling(False)
        assert m.numerics_flags(clear=True) == 0
    finally:
        m.close()
    assert n_tail == (4 if B <= 16 else 0), n_tail
    l2 = waypoint_l2(out["trajectory"].numpy(), ref["trajectory"].numpy())
    _report([f"== small-batch forms at B={B}: waypoint L2 vs oracle {l2:.3e}, gpt_tail launches {n_tail}"])
    assert l2 <= WAYPOINT_L2_TOL


@pytest.mark.gpu
def test_decoder_query_groups_are_bit_identical(gpu_model, seeded_sd, monkeypatch):
    """decoder_mk splits a scene's 20 modes over 4 (or 2) workgroups of 5 (10) queries (the default while B x 4 fits
    the chip); the last group to arrive at the scene's counter runs the mode selection and the next taps' dedup.
    Every row's arithmetic is the same as in the one-workgroup form (DDMI_MK_GROUPS=1): the outputs, the selected
    modes and the graph replays (the counters reset themselves) are bit-identical."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    B = 3
    inp = synthetic_inputs(B, 61)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"]).cuda()

    def run(groups):
        monkeypatch.setenv("DDMI_MK_GROUPS", groups)
        m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
        try:
            outs = [{k: v.cpu().numpy() for k, v in m.forward(feats, noise=nz, modes=True).items()} for _ in range(3)]
        finally:
            m.close()
        return outs

    ref = run("1")
    for g in ("2", "4"):
        outs = run(g)
        for o in outs:
            for k in ref[0]:
                assert np.array_equal(o[k], ref[0][k]), (g, k)


@pytest.mark.gpu
@pytest.mark.parametrize("B,streams", [(8, 2), (8, 1), (64, 2)])
def test_replays_are_deterministic_across_inputs(seeded_sd, B, streams):
    """Every inter-workgroup hand-off of the forward (the tf decoder's exchanges at small batches, the decoder's query
    groups, the union value_proj's K splits) leaves its scratch holding the last batch's values: a stale read would
    show as a replay that differs from the same inputs' first run. Four input sets, each run twice with the other
    sets in between, on one handle (captured graphs, replays): every replay bit-identical to its input set's first
    run, with its query_out / agent K|V taps, and no flag raised."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    try:
        m.set_streams(streams)
        first = {}
        for rep in range(2):
            for s in (310, 311, 312, 313):
                inp = synthetic_inputs(B, s)
                f = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
                out = m.forward(f, noise=torch.from_numpy(inp["noise"]), modes=True)
                got = {k: v.cpu().numpy().copy() for k, v in out.items()}
                got["query_out"] = m.tap("query_out").cpu().numpy()[: B * 31 * 256].copy()
                got["agent_kv0"] = m.tap("agent_kv0").cpu().numpy()[: B * 30 * 512].copy()
                assert m.numerics_flags(clear=True) == 0, (s, rep)
                if rep == 0:
                    first[s] = got
                    continue
                bad = {k: float(np.abs(v - first[s][k]).max()) for k, v in got.items() if not np.array_equal(v, first[s][k])}
                assert not bad, (B, streams, s, bad)
    finally:
        m.close()
