"""CPU ORACLE — test infrastructure, never the product.

A functional fp32 PyTorch-CPU restatement of DiffusionDrive's inference forward
(``V2TransfuserModel.forward`` in eval mode), written from the reference's algorithm and
operating directly on a state dict in the reference key schema. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and only
as the checker / CPU baseline. The product path (``diffusiondrive_amd``) never calls it.

Pinned by ``tests/golden/*.npz``: goldens produced by importing the reference itself
(``/root/reference``) in the build container with offline shims for timm / diffusers /
nuplan (``tests/golden/make_golden.py``). timm and diffusers are unpinned third-party
dependencies absent here; their arithmetic is restated in ``tests/golden/refshim`` and in
this file.
"""
import math
from typing import Dict, Mapping, Optional

import numpy as np
import torch
import torch.nn.functional as F

from diffusiondrive_amd.config import TransfuserConfig, trunk_blocks

BN_EPS = 1e-5
LN_EPS = 1e-5


class Taps(dict):
    """Optional recorder of named intermediates (for debugging and per-stage parity)."""

    def put(self, name, t):
        self[name] = t.detach().clone()


def _t(sd, k):
    return sd[k]


# --------------------------------------------------------------------------- primitives
def bn(x, sd, p):
    """BatchNorm2d in eval mode (running stats), timm resnet bn*/downsample.1."""
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], False, 0.0, BN_EPS)


def linear(x, sd, p, bias=True):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"] if bias else None)


def layer_norm(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], LN_EPS)


def conv(x, sd, p, stride=1, padding=0, bias=False):
    return F.conv2d(x, sd[p + ".weight"], sd[p + ".bias"] if bias else None, stride, padding)


def mish(x):
    return x * torch.tanh(F.softplus(x))


def mha(q_in, kv_in, sd, p, nhead):
    """nn.MultiheadAttention(batch_first=True) forward, no mask, eval
    (used at transfuser_model_v2.py:73-82 via nn.TransformerDecoderLayer and :316-327)."""
    w, b = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
    d = q_in.shape[-1]
    q = F.linear(q_in, w[:d], b[:d])
    k = F.linear(kv_in, w[d:2 * d], b[d:2 * d])
    v = F.linear(kv_in, w[2 * d:], b[2 * d:])
    B, Lq, _ = q.shape
    Lk = k.shape[1]
    hd = d // nhead
    q = q.view(B, Lq, nhead, hd).transpose(1, 2)
    k = k.view(B, Lk, nhead, hd).transpose(1, 2)
    v = v.view(B, Lk, nhead, hd).transpose(1, 2)
    att = torch.softmax((q @ k.transpose(-2, -1)) / math.sqrt(hd), dim=-1)
    y = (att @ v).transpose(1, 2).reshape(B, Lq, d)
    return linear(y, sd, p + ".out_proj")


# --------------------------------------------------------------------------- backbone
def trunk_stem(x, sd, p):
    """timm ResNet stem conv1/bn1/act1 (transfuser_backbone.py:180-185)."""
    return F.relu(bn(conv(x, sd, p + ".conv1", 2, 3), sd, p + ".bn1"))


def trunk_layer(x, sd, p, arch, i):
    """maxpool (before layer1) + layer{i+1} BasicBlocks/Bottlenecks (transfuser_backbone.py:188-192)."""
    kind, layers = trunk_blocks(arch)
    if i == 0:
        x = F.max_pool2d(x, 3, 2, 1)
    for b in range(layers[i]):
        q = f"{p}.layer{i + 1}.{b}"
        stride = 2 if (b == 0 and i > 0) else 1
        sc = x
        if kind == "basic":
            y = F.relu(bn(conv(x, sd, q + ".conv1", stride, 1), sd, q + ".bn1"))
            y = bn(conv(y, sd, q + ".conv2", 1, 1), sd, q + ".bn2")
        else:
            y = F.relu(bn(conv(x, sd, q + ".conv1"), sd, q + ".bn1"))
            y = F.relu(bn(conv(y, sd, q + ".conv2", stride, 1), sd, q + ".bn2"))
            y = bn(conv(y, sd, q + ".conv3"), sd, q + ".bn3")
        if (q + ".downsample.0.weight") in sd:
            sc = bn(conv(x, sd, q + ".downsample.0", stride), sd, q + ".downsample.1")
        x = F.relu(y + sc)
    return x


def gpt(img, lid, sd, p, cfg):
    """GPT fusion (transfuser_backbone.py:327-362, Block :427-431, SelfAttention :385-409)."""
    B, C, ih, iw = img.shape
    lh, lw = lid.shape[2:]
    tok = torch.cat([img.permute(0, 2, 3, 1).reshape(B, -1, C),
                     lid.permute(0, 2, 3, 1).reshape(B, -1, C)], 1)
    x = sd[p + ".pos_emb"] + tok
    nh = cfg.n_head
    hs = C // nh
    for b in range(cfg.n_layer):
        q = f"{p}.blocks.{b}"
        h = layer_norm(x, sd, q + ".ln1")
        T = h.shape[1]
        kk = linear(h, sd, q + ".attn.key").view(B, T, nh, hs).transpose(1, 2)
        qq = linear(h, sd, q + ".attn.query").view(B, T, nh, hs).transpose(1, 2)
        vv = linear(h, sd, q + ".attn.value").view(B, T, nh, hs).transpose(1, 2)
        att = torch.softmax((qq @ kk.transpose(-2, -1)) * (1.0 / math.sqrt(hs)), dim=-1)
        y = (att @ vv).transpose(1, 2).reshape(B, T, C)
        x = x + linear(y, sd, q + ".attn.proj")
        h = layer_norm(x, sd, q + ".ln2")
        x = x + linear(F.relu(linear(h, sd, q + ".mlp.0")), sd, q + ".mlp.2")
    x = layer_norm(x, sd, p + ".ln_f")
    n_img = ih * iw
    img_o = x[:, :n_img].reshape(B, ih, iw, C).permute(0, 3, 1, 2)
    lid_o = x[:, n_img:].reshape(B, lh, lw, C).permute(0, 3, 1, 2)
    return img_o, lid_o


def fuse(img, lid, sd, i, cfg):
    """TransfuserBackbone.fuse_features (transfuser_backbone.py:241-276)."""
    ie = F.adaptive_avg_pool2d(img, (cfg.img_vert_anchors, cfg.img_horz_anchors))
    le = F.adaptive_avg_pool2d(lid, (cfg.lidar_vert_anchors, cfg.lidar_horz_anchors))
    le = conv(le, sd, f"_backbone.lidar_channel_to_img.{i}", bias=True)
    io, lo = gpt(ie, le, sd, f"_backbone.transformers.{i}", cfg)
    lo = conv(lo, sd, f"_backbone.img_channel_to_lidar.{i}", bias=True)
    io = F.interpolate(io, size=img.shape[2:], mode="bilinear", align_corners=False)
    lo = F.interpolate(lo, size=lid.shape[2:], mode="bilinear", align_corners=False)
    return img + io, lid + lo


def backbone(cam, lidar, sd, cfg, taps: Optional[Taps] = None):
    """TransfuserBackbone.forward with transformer_decoder_join=True (transfuser_backbone.py:161-224)."""
    img = trunk_stem(cam, sd, "_backbone.image_encoder")
    lid = trunk_stem(lidar, sd, "_backbone.lidar_encoder")
    for i in range(4):
        img = trunk_layer(img, sd, "_backbone.image_encoder", cfg.image_architecture, i)
        lid = trunk_layer(lid, sd, "_backbone.lidar_encoder", cfg.lidar_architecture, i)
        if taps is not None:
            taps.put(f"img_l{i + 1}", img)
            taps.put(f"lid_l{i + 1}", lid)
        img, lid = fuse(img, lid, sd, i, cfg)
        if taps is not None:
            taps.put(f"img_f{i + 1}", img)
            taps.put(f"lid_f{i + 1}", lid)
    # top_down (:153-159)
    p5 = F.relu(conv(lid, sd, "_backbone.c5_conv", bias=True))
    p4 = F.interpolate(p5, scale_factor=cfg.bev_upsample_factor, mode="bilinear", align_corners=False)
    p4 = F.relu(conv(p4, sd, "_backbone.up_conv5", 1, 1, bias=True))
    hw = (cfg.lidar_resolution_height // cfg.bev_down_sample_factor,
          cfg.lidar_resolution_width // cfg.bev_down_sample_factor)
    p3 = F.interpolate(p4, size=hw, mode="bilinear", align_corners=False)
    p3 = F.relu(conv(p3, sd, "_backbone.up_conv4", 1, 1, bias=True))
    return p3, lid


# --------------------------------------------------------------------------- trajectory head
def norm_odo(x):
    """TrajectoryHead.norm_odo on (...,2) input (transfuser_model_v2.py:480-489)."""
    return torch.stack([2 * (x[..., 0] + 1.2) / 56.9 - 1, 2 * (x[..., 1] + 20) / 46 - 1], -1)


def denorm_odo(x):
    """TrajectoryHead.denorm_odo on (...,2) input (transfuser_model_v2.py:491-500)."""
    return torch.stack([(x[..., 0] + 1) / 2 * 56.9 - 1.2, (x[..., 1] + 1) / 2 * 46 - 20], -1)


def sine_embed(pos, hidden_dim=64):
    """gen_sineembed_for_position (blocks.py:22-40): output cat(pos_y, pos_x)."""
    half = hidden_dim // 2
    dim_t = torch.arange(half, dtype=torch.float32)
    dim_t = 10000 ** (2 * (dim_t // 2) / half)
    xe = pos[..., 0] * (2 * math.pi)
    ye = pos[..., 1] * (2 * math.pi)
    px = xe[..., None] / dim_t
    py = ye[..., None] / dim_t
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), -1).flatten(-2)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), -1).flatten(-2)
    return torch.cat((py, px), -1)


def timestep_embed(t, dim=256):
    """SinusoidalPosEmb (conditional_unet1d.py:53-66) for an int64 timestep vector."""
    half = dim // 2
    e = math.log(10000) / (half - 1)
    e = torch.exp(torch.arange(half) * -e)
    e = t[:, None] * e[None, :]
    return torch.cat((e.sin(), e.cos()), -1)


class DDIM:
    """diffusers DDIMScheduler restated for the reference's use (transfuser_model_v2.py:447-451;
    add_noise :595-597; step eta=0, prediction_type='sample', clip_sample=True :634-636)."""

    def __init__(self, num_train=1000, beta_start=1e-4, beta_end=0.02):
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train, dtype=torch.float32) ** 2
        self.num_train = num_train
        self.ac = torch.cumprod(1.0 - betas, 0)
        self.final = torch.tensor(1.0)

    def add_noise(self, x0, noise, t):
        a = self.ac[t]
        return a ** 0.5 * x0 + (1 - a) ** 0.5 * noise

    def step(self, x0, t, sample, num_inference):
        # forward_test calls set_timesteps(1000) (:584), so prev_t = t - 1000 // 1000 = t - 1.
        prev = t - self.num_train // num_inference
        a_t = self.ac[t]
        a_p = self.ac[prev] if prev >= 0 else self.final
        b_t = 1 - a_t
        eps = (sample - a_t ** 0.5 * x0) / b_t ** 0.5
        x0c = x0.clamp(-1.0, 1.0)
        return a_p ** 0.5 * x0c + (1 - a_p) ** 0.5 * eps


def grid_sample_attention(query, points, bev, sd, p, cfg, value=None, taps=None, tag=""):
    """GridSampleCrossBEVAttention.forward (blocks.py:88-129)."""
    B, Q, P, _ = points.shape
    g = torch.stack([points[..., 1] / cfg.lidar_max_x, points[..., 0] / cfg.lidar_max_y], -1)
    w = torch.softmax(linear(query, sd, p + ".attention_weights").view(B, Q, P), -1)
    if value is None:
        value = F.relu(conv(bev, sd, p + ".value_proj.0", 1, 1, bias=True))
    s = F.grid_sample(value, g, mode="bilinear", padding_mode="zeros", align_corners=False)
    out = (w.unsqueeze(1) * s).sum(-1).permute(0, 2, 1)
    if taps is not None:
        taps.put(f"gs_{tag}", out)
    return linear(out, sd, p + ".output_proj") + query


def diff_layer(x, pts, bev, agents, ego, temb, sd, p, cfg, value, taps=None, tag=""):
    """CustomTransformerDecoderLayer.forward (transfuser_model_v2.py:343-382)."""
    x = grid_sample_attention(x, pts, bev, sd, p + ".cross_bev_attention", cfg, value, taps, tag)
    x = layer_norm(x + mha(x, agents, sd, p + ".cross_agent_attention", cfg.tf_num_head), sd, p + ".norm1")
    x = layer_norm(x + mha(x, ego, sd, p + ".cross_ego_attention", cfg.tf_num_head), sd, p + ".norm2")
    x = layer_norm(linear(F.relu(linear(x, sd, p + ".ffn.0")), sd, p + ".ffn.2"), sd, p + ".norm3")
    ss = linear(mish(temb), sd, p + ".time_modulation.scale_shift_mlp.1")
    scale, shift = ss.chunk(2, -1)
    x = x * (1 + scale) + shift
    t = p + ".task_decoder"
    c = layer_norm(F.relu(linear(x, sd, t + ".plan_cls_branch.0")), sd, t + ".plan_cls_branch.2")
    c = layer_norm(F.relu(linear(c, sd, t + ".plan_cls_branch.3")), sd, t + ".plan_cls_branch.5")
    cls = linear(c, sd, t + ".plan_cls_branch.6").squeeze(-1)
    r = F.relu(linear(x, sd, t + ".plan_reg_branch.0"))
    r = F.relu(linear(r, sd, t + ".plan_reg_branch.2"))
    r = linear(r, sd, t + ".plan_reg_branch.4").reshape(x.shape[0], x.shape[1], -1, 3)
    reg = torch.cat([r[..., :2] + pts, (torch.tanh(r[..., 2:3]) * np.pi)], -1)
    return reg, cls


def trajectory_head(ego_q, agents_q, bev, sd, cfg, noise, steps=None, taps=None, schedule="truncated"):
    """TrajectoryHead.forward_test (transfuser_model_v2.py:578-641). ``steps`` generalises the
    hard-coded step_num=2 (:581) for the C5 latency ablation; steps=2 is the reference.
    ``schedule="vanilla"`` is the C5 ablation's non-truncated DDIM (no reference counterpart):
    x_T = noise and diffusers' "leading" set_timesteps(steps) over the 1000 train steps."""
    steps = steps or cfg.denoise_steps
    p = "_trajectory_head"
    B = ego_q.shape[0]
    sched = DDIM(cfg.num_train_timesteps)
    if schedule == "vanilla":
        step_ratio = cfg.num_train_timesteps // steps
        roll = (np.arange(0, steps) * step_ratio)[::-1].copy().astype(np.int64)
        img = noise.clone()
        num_inference = steps
    else:
        ratio = cfg.step_span / steps
        roll = (np.arange(0, steps) * ratio).round()[::-1].copy().astype(np.int64)
        anchor = sd[p + ".plan_anchor"].unsqueeze(0).repeat(B, 1, 1, 1)
        img = sched.add_noise(norm_odo(anchor), noise, cfg.trunc_timestep)
        num_inference = cfg.num_train_timesteps
    # value_proj depends only on layer weights + the BEV map: hoisted per layer (exact).
    values = [F.relu(conv(bev, sd, f"{p}.diff_decoder.layers.{l}.cross_bev_attention.value_proj.0", 1, 1, bias=True))
              for l in range(cfg.num_diff_layers)]
    reg = cls = None
    for si, k in enumerate(roll):
        x = torch.clamp(img, -1, 1)
        pts = denorm_odo(x)
        emb = sine_embed(pts, 64).flatten(-2)
        tf = linear(emb, sd, p + ".plan_anchor_encoder.0")
        tf = layer_norm(F.relu(tf), sd, p + ".plan_anchor_encoder.2")
        tf = linear(tf, sd, p + ".plan_anchor_encoder.3")
        te = timestep_embed(torch.full((B,), int(k), dtype=torch.int64))
        te = linear(mish(linear(te, sd, p + ".time_mlp.1")), sd, p + ".time_mlp.3").view(B, 1, -1)
        cur = pts
        for l in range(cfg.num_diff_layers):
            reg, cls = diff_layer(tf, cur, bev, agents_q, ego_q, te, sd,
                                  f"{p}.diff_decoder.layers.{l}", cfg, values[l], taps, f"s{si}l{l}")
            if taps is not None:
                taps.put(f"reg_s{si}l{l}", reg)
                taps.put(f"cls_s{si}l{l}", cls)
            cur = reg[..., :2]
        img = sched.step(norm_odo(reg[..., :2]), int(k), img, num_inference)
    idx = cls.argmax(-1)
    best = reg[torch.arange(B), idx]
    return best, reg, cls


def trajectory_head_train(ego_q, agents_q, bev, sd, cfg, noise, timesteps, taps=None):
    """TrajectoryHead.forward_train (transfuser_model_v2.py:520-576) with its two random draws passed in
    (``timesteps`` ~ randint(0, 50) (B,), ``noise`` ~ randn (B, 20, 8, 2), :533-534): per-scene truncated noise
    on the normalised plan anchors, clamp, denorm, ONE pass of the cascade decoder with the per-scene time
    embedding (:537-556). Returns (best_reg, [reg per layer], [cls per layer])."""
    p = "_trajectory_head"
    B = ego_q.shape[0]
    sched = DDIM(cfg.num_train_timesteps)
    anchor = sd[p + ".plan_anchor"].unsqueeze(0).repeat(B, 1, 1, 1)
    t = torch.as_tensor(timesteps).to(torch.int64)
    a = sched.ac[t].view(B, 1, 1, 1)
    noisy = a ** 0.5 * norm_odo(anchor) + (1 - a) ** 0.5 * noise
    pts = denorm_odo(torch.clamp(noisy.float(), -1, 1))
    emb = sine_embed(pts, 64).flatten(-2)
    tf = linear(emb, sd, p + ".plan_anchor_encoder.0")
    tf = layer_norm(F.relu(tf), sd, p + ".plan_anchor_encoder.2")
    tf = linear(tf, sd, p + ".plan_anchor_encoder.3")
    te = timestep_embed(t)
    te = linear(mish(linear(te, sd, p + ".time_mlp.1")), sd, p + ".time_mlp.3").view(B, 1, -1)
    values = [F.relu(conv(bev, sd, f"{p}.diff_decoder.layers.{l}.cross_bev_attention.value_proj.0", 1, 1, bias=True))
              for l in range(cfg.num_diff_layers)]
    regs, clss = [], []
    cur = pts
    for l in range(cfg.num_diff_layers):
        reg, cls = diff_layer(tf, cur, bev, agents_q, ego_q, te, sd, f"{p}.diff_decoder.layers.{l}", cfg, values[l],
                              taps, f"train_l{l}")
        regs.append(reg)
        clss.append(cls)
        cur = reg[..., :2]
    idx = clss[-1].argmax(-1)
    return regs[-1][torch.arange(B), idx], regs, clss


def sigmoid_focal_loss(pred, target, gamma=2.0, alpha=0.25):
    """py_sigmoid_focal_loss (multimodal_loss.py:71-114), reduction 'mean', no weight."""
    ps = pred.sigmoid()
    target = target.type_as(pred)
    pt = (1 - ps) * target + ps * (1 - target)
    fw = (alpha * target + (1 - alpha) * (1 - target)) * pt.pow(gamma)
    return (F.binary_cross_entropy_with_logits(pred, target, reduction="none") * fw).mean()


def loss_computer(reg, cls, target_traj, anchor, cfg):
    """LossComputer.forward (multimodal_loss.py:131-168): the anchor mode nearest the target (mean over poses of
    the xy distance) is the class target of a focal loss over the 20 logits and selects the regressed
    trajectory of an L1 loss against the target (all 3 channels)."""
    B, M, T, D = reg.shape
    dist = torch.linalg.norm(target_traj.unsqueeze(1)[..., :2] - anchor, dim=-1).mean(-1)
    mode = dist.argmin(-1)
    best = reg[torch.arange(B), mode]
    onehot = torch.zeros(B, M, dtype=cls.dtype)
    onehot[torch.arange(B), mode] = 1
    return (cfg.trajectory_cls_weight * sigmoid_focal_loss(cls, onehot)
            + cfg.trajectory_reg_weight * F.l1_loss(best, target_traj))


def agent_loss(targets, pred, cfg):
    """_agent_loss (transfuser_loss.py:54-113): BCE + L1 costs, Hungarian matching per scene (scipy, on CPU as
    the reference), then the matched box L1 over the valid targets and the label BCE."""
    from scipy.optimize import linear_sum_assignment
    gt_states = torch.as_tensor(targets["agent_states"])
    gt_valid = torch.as_tensor(targets["agent_labels"]).bool()
    ps, pl = pred["agent_states"], pred["agent_labels"]
    if cfg.latent:
        rad = torch.arctan2(gt_states[..., 1], gt_states[..., 0])
        gt_valid = gt_valid & (-cfg.latent_rad_thresh <= rad) & (rad <= cfg.latent_rad_thresh)
    B, N = ps.shape[:2]
    n_gt = gt_valid.sum()
    n_gt = n_gt if n_gt > 0 else n_gt + 1
    gv = gt_valid[:, :, None].float()
    pe = pl[:, None, :]
    mx = torch.relu(-pe)
    ce = ((1 - gv) * pe + mx + torch.log(torch.exp(-mx) + torch.exp(-pe - mx))).permute(0, 2, 1)
    l1 = (gt_valid[..., None].float() * (gt_states[:, :, None, :2] - ps[:, None, :, :2]).abs().sum(-1)).permute(0, 2, 1)
    cost = cfg.agent_class_weight * ce + cfg.agent_box_weight * l1
    src, dst = [], []
    for b in range(B):
        i, j = linear_sum_assignment(cost[b].numpy())
        src.append(torch.as_tensor(i, dtype=torch.int64))
        dst.append(torch.as_tensor(j, dtype=torch.int64))
    bidx = torch.cat([torch.full_like(s_, b) for b, s_ in enumerate(src)])
    sidx = torch.cat(src)
    gs_ = torch.cat([gt_states[b][j] for b, j in enumerate(dst)])
    gvl = torch.cat([gt_valid[b][j] for b, j in enumerate(dst)]).float()
    box = (F.l1_loss(ps[bidx, sidx], gs_, reduction="none").sum(-1) * gvl).view(B, -1).sum() / n_gt
    cls = F.binary_cross_entropy_with_logits(pl[bidx, sidx], gvl, reduction="none").view(B, -1).mean()
    return cls, box


def transfuser_loss(targets, pred, cfg):
    """transfuser_loss (transfuser_loss.py:11-51): weighted sum of the trajectory loss (forward_train's, else L1 of
    the trajectory), the agent class / box losses and the BEV semantic cross entropy."""
    if "trajectory_loss" in pred:
        traj = pred["trajectory_loss"]
    else:
        traj = F.l1_loss(pred["trajectory"], torch.as_tensor(targets["trajectory"]))
    ac, ab = agent_loss(targets, pred, cfg)
    bev = F.cross_entropy(pred["bev_semantic_map"], torch.as_tensor(targets["bev_semantic_map"]).long())
    diff = pred.get("diffusion_loss", 0)
    out = {"loss": cfg.trajectory_weight * traj + cfg.diff_loss_weight * diff + cfg.agent_class_weight * ac
           + cfg.agent_box_weight * ab + cfg.bev_semantic_weight * bev,
           "trajectory_loss": cfg.trajectory_weight * traj, "diffusion_loss": cfg.diff_loss_weight * diff,
           "agent_class_loss": cfg.agent_class_weight * ac, "agent_box_loss": cfg.agent_box_weight * ab,
           "bev_semantic_loss": cfg.bev_semantic_weight * bev}
    out.update(pred.get("trajectory_loss_dict", {}))
    return out


# --------------------------------------------------------------------------- full model
class OracleModel:
    """fp32 CPU restatement of V2TransfuserModel.forward in eval mode (transfuser_model_v2.py:98-162)."""

    def __init__(self, state_dict: Mapping[str, np.ndarray], cfg: TransfuserConfig = None):
        self.cfg = cfg or TransfuserConfig()
        self.sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}

    @torch.no_grad()
    def forward(self, camera, lidar, status, noise, steps=None, taps: Optional[Taps] = None,
                heads=True, schedule="truncated") -> Dict[str, torch.Tensor]:
        nz = torch.as_tensor(np.asarray(noise))
        ego_q, agents_q, cross, p3 = self._features(camera, lidar, status, taps)
        traj, reg, cls = trajectory_head(ego_q, agents_q, cross, self.sd, self.cfg, nz, steps, taps, schedule)
        out = {"trajectory": traj, "poses_reg": reg, "poses_cls": cls}
        if heads:
            out.update(self._heads(p3, agents_q))
        return out

    @torch.no_grad()
    def forward_train(self, camera, lidar, status, noise, timesteps, targets, taps: Optional[Taps] = None,
                      heads=True) -> Dict[str, torch.Tensor]:
        """V2TransfuserModel.forward with targets and the trajectory head in training mode (forward_train,
        transfuser_model_v2.py:520-576), the rest of the network in eval mode (the deterministic loss evaluator):
        ``trajectory``, ``trajectory_loss`` (sum over layers), ``trajectory_loss_dict``, the per-layer
        ``poses_reg_list`` / ``poses_cls_list`` and, with ``heads``, the BEV-semantic / agent outputs."""
        cfg, sd = self.cfg, self.sd
        nz = torch.as_tensor(np.asarray(noise))
        ego_q, agents_q, cross, p3 = self._features(camera, lidar, status, taps)
        best, regs, clss = trajectory_head_train(ego_q, agents_q, cross, sd, cfg, nz, timesteps, taps)
        tt = torch.as_tensor(np.asarray(targets["trajectory"]))
        anchor = sd["_trajectory_head.plan_anchor"].unsqueeze(0).repeat(nz.shape[0], 1, 1, 1)
        d = {f"trajectory_loss_{i}": loss_computer(r, c, tt, anchor, cfg) for i, (r, c) in enumerate(zip(regs, clss))}
        out = {"trajectory": best, "trajectory_loss": sum(d.values()), "trajectory_loss_dict": d,
               "poses_reg_list": regs, "poses_cls_list": clss}
        if heads:
            out.update(self._heads(p3, agents_q))
        return out

    def _features(self, camera, lidar, status, taps=None):
        """Everything of V2TransfuserModel.forward before the trajectory head (transfuser_model_v2.py:104-158)."""
        cfg, sd = self.cfg, self.sd
        cam = torch.as_tensor(np.asarray(camera))
        lid = torch.as_tensor(np.asarray(lidar))
        st = torch.as_tensor(np.asarray(status))
        B = st.shape[0]
        p3, bev = backbone(cam, lid, sd, cfg, taps)
        bev_tok = conv(bev, sd, "_bev_downscale", bias=True).flatten(-2).permute(0, 2, 1)
        stat = linear(st, sd, "_status_encoding")
        keyval = torch.cat([bev_tok, stat[:, None]], 1) + sd["_keyval_embedding.weight"][None]
        ccb = keyval[:, :-1].permute(0, 2, 1).reshape(B, -1, bev.shape[2], bev.shape[3])
        ccb = F.interpolate(ccb, size=p3.shape[2:], mode="bilinear", align_corners=False)
        cross = torch.cat([ccb, p3], 1).flatten(-2).permute(0, 2, 1)
        cross = layer_norm(F.relu(linear(cross, sd, "bev_proj.0")), sd, "bev_proj.2")
        cross = cross.permute(0, 2, 1).reshape(B, -1, p3.shape[2], p3.shape[3])
        q = sd["_query_embedding.weight"][None].repeat(B, 1, 1)
        for i in range(cfg.tf_num_layers):
            pp = f"_tf_decoder.layers.{i}"
            q = layer_norm(q + mha(q, q, sd, pp + ".self_attn", cfg.tf_num_head), sd, pp + ".norm1")
            q = layer_norm(q + mha(q, keyval, sd, pp + ".multihead_attn", cfg.tf_num_head), sd, pp + ".norm2")
            ff = linear(F.relu(linear(q, sd, pp + ".linear1")), sd, pp + ".linear2")
            q = layer_norm(q + ff, sd, pp + ".norm3")
        if taps is not None:
            taps.put("p3", p3)
            taps.put("bev_feature", bev)
            taps.put("keyval", keyval)
            taps.put("cross_bev", cross)
            taps.put("query_out", q)
        return q[:, :1], q[:, 1:], cross, p3

    def _heads(self, p3, agents_q):
        """_bev_semantic_head and AgentHead (transfuser_model_v2.py:144,159,165-205)."""
        cfg, sd = self.cfg, self.sd
        out = {}
        h = F.relu(conv(p3, sd, "_bev_semantic_head.0", 1, 1, bias=True))
        h = conv(h, sd, "_bev_semantic_head.2", bias=True)
        out["bev_semantic_map"] = F.interpolate(
            h, size=(cfg.lidar_resolution_height // 2, cfg.lidar_resolution_width),
            mode="bilinear", align_corners=False)
        a = linear(F.relu(linear(agents_q, sd, "_agent_head._mlp_states.0")), sd, "_agent_head._mlp_states.2")
        # BoundingBox2DIndex: POINT = 0:2, HEADING = 2 (transfuser_features.py:388-443)
        a = torch.cat([torch.tanh(a[..., :2]) * 32, torch.tanh(a[..., 2:3]) * np.pi, a[..., 3:]], -1)
        out["agent_states"] = a
        out["agent_labels"] = linear(agents_q, sd, "_agent_head._mlp_label.0").squeeze(-1)
        return out
