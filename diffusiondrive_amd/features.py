"""Input feature builder (the input side of the boundary).

Mirrors ``TransfuserFeatureBuilder`` (transfuser_features.py:25-138) so ``compute_trajectory``
works end to end on an ``AgentInput``:

* camera: l0 / f0 / r0 crops [28:-28, 416:-416] / [28:-28] stitched side by side, resized to
  1024x256 with OpenCV ``INTER_LINEAR`` semantics, ``ToTensor`` (HWC uint8 -> CHW float / 255).
  cv2 is not installed here; for uint8 input and an exact integer down-scale factor f (the NAVSIM
  case: 4096x1024 -> 1024x256, f = 4) cv2's fixed-point INTER_LINEAR reduces to
  ``floor((p00 + p01 + p10 + p11 + 2) / 4)`` over the 2x2 source block at ``f*d + f/2 - 1``
  (coefficients 0.5/0.5 in Q11, final shift 22 with rounding), which is what this computes.
  Other sizes use a float bilinear resize (parity vs cv2 unpinned there).
* LiDAR: ``np.histogramdd`` splat of points with z in (0.2, 100) over 256x256 bins of
  [-32, 32] m, clipped at 5, divided by 5 (transfuser_features.py:79-138).
* status: [driving_command one-hot (4), ego_velocity (2), ego_acceleration (2)] (:46-53).
"""
from typing import Dict

import numpy as np
import torch

from .config import TransfuserConfig


def _resize_linear_uint8(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    h, w = img.shape[:2]
    if img.dtype == np.uint8 and h % out_h == 0 and w % out_w == 0 and h // out_h == w // out_w \
            and (h // out_h) % 2 == 0:
        f = h // out_h
        o = f // 2 - 1
        a = img[o::f][:out_h].astype(np.int32)
        b = img[o + 1::f][:out_h].astype(np.int32)
        s = a[:, o::f][:, :out_w] + a[:, o + 1::f][:, :out_w] + b[:, o::f][:, :out_w] + b[:, o + 1::f][:, :out_w]
        return ((s + 2) >> 2).astype(np.uint8)
    # generic float bilinear, align_corners=False (cv2 INTER_LINEAR geometry)
    x = img.astype(np.float32)
    ys = np.clip((np.arange(out_h) + 0.5) * h / out_h - 0.5, 0, h - 1)
    xs = np.clip((np.arange(out_w) + 0.5) * w / out_w - 0.5, 0, w - 1)
    y0, x0 = np.floor(ys).astype(int), np.floor(xs).astype(int)
    y1, x1 = np.minimum(y0 + 1, h - 1), np.minimum(x0 + 1, w - 1)
    ly, lx = (ys - y0)[:, None, None], (xs - x0)[None, :, None]
    r = (x[y0][:, x0] * (1 - lx) + x[y0][:, x1] * lx) * (1 - ly) + (x[y1][:, x0] * (1 - lx) + x[y1][:, x1] * lx) * ly
    return np.clip(np.rint(r), 0, 255).astype(np.uint8) if img.dtype == np.uint8 else r


def camera_feature(cam_l0: np.ndarray, cam_f0: np.ndarray, cam_r0: np.ndarray, cfg: TransfuserConfig) -> torch.Tensor:
    l0 = cam_l0[28:-28, 416:-416]
    f0 = cam_f0[28:-28]
    r0 = cam_r0[28:-28, 416:-416]
    stitched = np.concatenate([l0, f0, r0], axis=1)
    resized = _resize_linear_uint8(stitched, cfg.camera_width, cfg.camera_height)
    t = torch.from_numpy(np.ascontiguousarray(resized.transpose(2, 0, 1)))
    return t.float().div(255.0) if resized.dtype == np.uint8 else t.float()


def lidar_feature(points_xyz: np.ndarray, cfg: TransfuserConfig) -> torch.Tensor:
    """points_xyz: (N, 3) ego-frame points."""
    pc = points_xyz[points_xyz[..., 2] < cfg.max_height_lidar]
    above = pc[pc[..., 2] > cfg.lidar_split_height]

    def splat(p):
        nx = int((cfg.lidar_max_x - cfg.lidar_min_x) * int(cfg.pixels_per_meter)) + 1
        ny = int((cfg.lidar_max_y - cfg.lidar_min_y) * int(cfg.pixels_per_meter)) + 1
        xb = np.linspace(cfg.lidar_min_x, cfg.lidar_max_x, nx)
        yb = np.linspace(cfg.lidar_min_y, cfg.lidar_max_y, ny)
        hist = np.histogramdd(p[:, :2], bins=(xb, yb))[0]
        hist[hist > cfg.hist_max_per_pixel] = cfg.hist_max_per_pixel
        return hist / cfg.hist_max_per_pixel

    feats = [splat(above)]
    if cfg.use_ground_plane:
        below = pc[pc[..., 2] <= cfg.lidar_split_height]
        feats = [splat(below), splat(above)]
    return torch.tensor(np.stack(feats, axis=0).astype(np.float32))


class TransfuserFeatureBuilder:
    """transfuser_features.py:25-55 (inference features only)."""

    def __init__(self, config: TransfuserConfig):
        self._config = config

    def get_unique_name(self) -> str:
        return "transfuser_feature"

    def compute_features(self, agent_input) -> Dict[str, torch.Tensor]:
        cams = agent_input.cameras[-1]
        ego = agent_input.ego_statuses[-1]
        lidar_pc = agent_input.lidars[-1].lidar_pc[0:3].T  # LidarIndex.POSITION (x, y, z)
        return {
            "camera_feature": camera_feature(cams.cam_l0.image, cams.cam_f0.image, cams.cam_r0.image, self._config),
            "lidar_feature": lidar_feature(lidar_pc, self._config),
            "status_feature": torch.concatenate([
                torch.tensor(ego.driving_command, dtype=torch.float32),
                torch.tensor(ego.ego_velocity, dtype=torch.float32),
                torch.tensor(ego.ego_acceleration, dtype=torch.float32),
            ]),
        }
