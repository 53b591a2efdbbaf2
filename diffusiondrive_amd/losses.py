"""The training loss of the reference agent (``TransfuserAgent.compute_loss`` -> ``transfuser_loss``,
transfuser_agent.py:127-134, transfuser_loss.py:11-113) over the outputs of the MI355X forward.

* ``trajectory_loss``: forward_train's (the LossComputer sum over both decoder layers, computed on the GPU by
  ``dd_forward_train``), or - for an eval-mode prediction - the L1 of the trajectory against the target, as the
  reference falls back to (:22-25);
* the agent class / box losses: Hungarian matching of the 30 predicted boxes to the 30 target slots per scene on
  the CPU with scipy's ``linear_sum_assignment``, exactly where the reference runs it (``cost.cpu()``, :89-91); the
  cost matrices and matched sums are (B, 30, 30) / (B, 30) host arithmetic;
* the BEV-semantic cross entropy (:28-29) on the GPU (``dd_bev_semantic_loss``, train_loss.hip).

The weights are the reference config's (TransfuserConfig :82-89). ``diffusion_loss`` is 0 as in the reference
(its predictions never carry one).
"""
import ctypes
from typing import Dict

import numpy as np
import torch

from . import _lib
from .config import TransfuserConfig


def _np(t):
    return t.detach().float().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t, np.float32)


def _bce_logits(x, t):
    """binary_cross_entropy_with_logits as ATen evaluates it (reduction none), float32."""
    x = x.astype(np.float32)
    t = t.astype(np.float32)
    mv = np.maximum(-x, np.float32(0))
    return (np.float32(1) - t) * x + mv + np.log(np.exp(-mv) + np.exp(-x - mv))


def agent_loss(targets: Dict, predictions: Dict, config: TransfuserConfig):
    """_agent_loss (transfuser_loss.py:54-113): BCE + L1 costs (:116-155), Hungarian matching per scene on the CPU
    (scipy), then the matched box L1 over the valid targets / n_gt and the label BCE mean."""
    from scipy.optimize import linear_sum_assignment
    gt_states = _np(targets["agent_states"])
    gt_valid = np.asarray(_np(targets["agent_labels"])).astype(bool)
    ps, pl = _np(predictions["agent_states"]), _np(predictions["agent_labels"])
    if config.latent:
        rad = np.arctan2(gt_states[..., 1], gt_states[..., 0])
        gt_valid = gt_valid & (-config.latent_rad_thresh <= rad) & (rad <= config.latent_rad_thresh)
    B, N = ps.shape[:2]
    n_gt = max(int(gt_valid.sum()), 1)
    gv = gt_valid[:, :, None].astype(np.float32)
    ce = _bce_logits(np.broadcast_to(pl[:, None, :], (B, N, N)), np.broadcast_to(gv, (B, N, N))).transpose(0, 2, 1)
    l1 = (gv * np.abs(gt_states[:, :, None, :2] - ps[:, None, :, :2]).sum(-1)).transpose(0, 2, 1)
    cost = np.float32(config.agent_class_weight) * ce + np.float32(config.agent_box_weight) * l1
    box_sum, bce = np.float32(0), []
    for b in range(B):
        i, j = linear_sum_assignment(cost[b])
        v = gt_valid[b][j].astype(np.float32)
        box_sum = box_sum + (np.abs(ps[b][i] - gt_states[b][j]).sum(-1) * v).sum(dtype=np.float32)
        bce.append(_bce_logits(pl[b][i], v))
    return float(np.mean(np.concatenate(bce))), float(box_sum / np.float32(n_gt))


def bev_semantic_loss(model, logits: torch.Tensor, target) -> torch.Tensor:
    """F.cross_entropy(bev_semantic_map, target.long()) on the GPU (dd_bev_semantic_loss)."""
    # eval-mode predictions come back on the CPU (the reference's contract); the loss runs on the model's device
    logits = torch.as_tensor(logits).to(device=f"cuda:{model.device}", dtype=torch.float32)
    B, C, H, W = logits.shape
    tg = torch.as_tensor(target)
    if tuple(tg.shape) != (B, H, W):
        raise ValueError(f"bev_semantic_map target must be (B,{H},{W}), got {tuple(tg.shape)}")
    # F.cross_entropy raises on a class id outside [0, C) (uint8 ids included); the kernel itself turns such an
    # id into a NaN loss rather than reading past the logits
    if tg.numel() and (int(tg.min()) < 0 or int(tg.max()) >= C):
        raise ValueError(f"bev_semantic_map target ids must lie in [0, {C})")
    if tg.dtype != torch.uint8:
        tg = tg.to(torch.uint8)
    tg = tg.to(logits.device).contiguous()
    lg = logits.contiguous()
    lib = model.lib
    work = torch.empty(int(lib.dd_bev_semantic_loss_work(B, H, W)), device=logits.device)
    out = torch.empty(1, device=logits.device)
    s = torch.cuda.current_stream(logits.device)
    _lib.check(lib.dd_bev_semantic_loss(lg.data_ptr(), tg.data_ptr(), B, C, H, W, work.data_ptr(), out.data_ptr(),
                                        ctypes.c_void_p(s.cuda_stream)), lib)
    return out[0]


def transfuser_loss(targets: Dict, predictions: Dict, config: TransfuserConfig, model) -> Dict[str, torch.Tensor]:
    """transfuser_loss (transfuser_loss.py:11-51): the weighted loss and its dict (0-d tensors)."""
    if "trajectory_loss" in predictions:
        traj = torch.as_tensor(predictions["trajectory_loss"]).float().cpu()
    else:
        d = _np(predictions["trajectory"]) - _np(targets["trajectory"])
        traj = torch.tensor(float(np.abs(d).mean(dtype=np.float32)))
    ac, ab = agent_loss(targets, predictions, config)
    ac, ab = torch.tensor(ac), torch.tensor(ab)
    bev = bev_semantic_loss(model, predictions["bev_semantic_map"], targets["bev_semantic_map"]).cpu()
    diff = torch.tensor(0.0)
    loss = (config.trajectory_weight * traj + config.diff_loss_weight * diff + config.agent_class_weight * ac
            + config.agent_box_weight * ab + config.bev_semantic_weight * bev)
    out = {"loss": loss, "trajectory_loss": config.trajectory_weight * traj,
           "diffusion_loss": config.diff_loss_weight * diff, "agent_class_loss": config.agent_class_weight * ac,
           "agent_box_loss": config.agent_box_weight * ab, "bev_semantic_loss": config.bev_semantic_weight * bev}
    for k, v in predictions.get("trajectory_loss_dict", {}).items():
        out[k] = torch.as_tensor(v).float().cpu()
    return out
