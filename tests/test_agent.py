"""Agent surface (drop-in boundary): feature builder on CPU, compute_trajectory on the GPU."""
from dataclasses import dataclass
from typing import List

import numpy as np
import pytest
import torch

from diffusiondrive_amd.config import TransfuserConfig


@dataclass
class _Cam:
    image: np.ndarray


@dataclass
class _Cams:
    cam_f0: _Cam
    cam_l0: _Cam
    cam_r0: _Cam


@dataclass
class _Lidar:
    lidar_pc: np.ndarray


@dataclass
class _Ego:
    ego_velocity: np.ndarray
    ego_acceleration: np.ndarray
    driving_command: np.ndarray


@dataclass
class _AgentInput:
    ego_statuses: List[_Ego]
    cameras: List[_Cams]
    lidars: List[_Lidar]


def make_agent_input(seed=0, n_points=20000):
    r = np.random.default_rng(seed)
    cams = _Cams(*(_Cam(r.integers(0, 256, (1080, 1920, 3), dtype=np.uint8)) for _ in range(3)))
    pts = np.zeros((6, n_points), np.float32)
    pts[0] = r.uniform(-40, 40, n_points)
    pts[1] = r.uniform(-40, 40, n_points)
    pts[2] = r.uniform(-1, 3, n_points)
    ego = _Ego(np.array([4.0, 0.3], np.float32), np.array([0.1, -0.2], np.float32), np.array([0, 1, 0, 0]))
    return _AgentInput([ego], [cams], [_Lidar(pts)])


def test_feature_builder_shapes_and_lidar_histogram():
    from diffusiondrive_amd.features import TransfuserFeatureBuilder
    cfg = TransfuserConfig()
    ai = make_agent_input()
    f = TransfuserFeatureBuilder(cfg).compute_features(ai)
    assert f["camera_feature"].shape == (3, 256, 1024) and f["camera_feature"].dtype == torch.float32
    assert f["lidar_feature"].shape == (1, 256, 256)
    assert torch.equal(f["status_feature"], torch.tensor([0, 1, 0, 0, 4.0, 0.3, 0.1, -0.2]))
    # LiDAR: independent restatement of the splat (transfuser_features.py:111-138)
    p = ai.lidars[-1].lidar_pc[:3].T
    p = p[(p[:, 2] < 100) & (p[:, 2] > 0.2)]
    inside = (p[:, 0] >= -32) & (p[:, 0] <= 32) & (p[:, 1] >= -32) & (p[:, 1] <= 32)
    ix = np.clip(np.floor((p[inside, 0] + 32) * 4).astype(int), 0, 255)
    iy = np.clip(np.floor((p[inside, 1] + 32) * 4).astype(int), 0, 255)
    h = np.zeros((256, 256))
    np.add.at(h, (ix, iy), 1)
    assert np.allclose(f["lidar_feature"][0].numpy(), np.minimum(h, 5) / 5)
    assert 0.0 <= float(f["camera_feature"].min()) and float(f["camera_feature"].max()) <= 1.0


def test_camera_resize_4x_matches_generic_bilinear():
    from diffusiondrive_amd.features import _resize_linear_uint8
    r = np.random.default_rng(1)
    img = r.integers(0, 256, (64, 256, 3), dtype=np.uint8)
    fast = _resize_linear_uint8(img, 64, 16).astype(int)
    ref = ((img[1::4, 1::4].astype(float) + img[1::4, 2::4] + img[2::4, 1::4] + img[2::4, 2::4]) / 4)
    assert np.abs(fast - ref).max() <= 0.5 + 1e-9  # round-half-up of the 2x2 mean


@pytest.mark.gpu
def test_compute_trajectory_matches_oracle(gpu, seeded_sd, tmp_path):
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    from diffusiondrive_amd.features import TransfuserFeatureBuilder
    from oracle.model import OracleModel
    ckpt = tmp_path / "dd.pth"
    torch.save({"state_dict": {"agent._transfuser_model." + k: torch.from_numpy(np.asarray(v))
                               for k, v in seeded_sd.items()}}, ckpt)
    agent = DiffusionDriveAgent(TransfuserConfig(), lr=1e-4, checkpoint_path=str(ckpt), device=0)
    ai = make_agent_input(3)
    torch.manual_seed(77)
    traj = agent.compute_trajectory(ai)
    assert traj.poses.shape == (8, 3) and traj.poses.dtype == np.float32
    f = TransfuserFeatureBuilder(TransfuserConfig()).compute_features(ai)
    torch.manual_seed(77)
    noise = torch.randn(1, 20, 8, 2)
    ref = OracleModel(seeded_sd).forward(f["camera_feature"][None], f["lidar_feature"][None],
                                         f["status_feature"][None], noise, heads=False)["trajectory"][0].numpy()
    l2 = float(np.sqrt(((traj.poses[:, :2].astype(np.float64) - ref[:, :2]) ** 2).sum()))
    assert l2 <= 1e-4, l2
    out = agent.forward({k: v[None] for k, v in f.items()}, noise=noise)
    assert set(out) >= {"trajectory", "bev_semantic_map", "agent_states", "agent_labels"}
    assert out["bev_semantic_map"].shape == (1, 7, 128, 256)
