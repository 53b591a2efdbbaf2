"""Hot-path constants of DiffusionDrive, mirrored from the reference's ``TransfuserConfig``.

Reference: ``navsim/agents/diffusiondrive/transfuser_config.py:10-149``. Only the fields the
inference forward reads are kept; training / loss / BEV-semantic-target fields are out of
scope. ``trajectory_sampling`` is a plain (num_poses, interval)
pair because nuplan is not available here.
"""
from dataclasses import dataclass, field
from typing import Optional


@dataclass(frozen=True)
class TrajectorySampling:
    """nuplan TrajectorySampling stand-in (transfuser_config.py:14-15)."""
    time_horizon: float = 4.0
    interval_length: float = 0.5

    @property
    def num_poses(self) -> int:
        return int(round(self.time_horizon / self.interval_length))


@dataclass
class TransfuserConfig:
    """Hyper-parameters of the DiffusionDrive inference path (transfuser_config.py:10-149)."""

    trajectory_sampling: TrajectorySampling = field(default_factory=TrajectorySampling)
    image_architecture: str = "resnet34"            # :17
    lidar_architecture: str = "resnet34"            # :18
    plan_anchor_path: Optional[str] = None          # :20 (anchors also live in the state_dict)

    lidar_min_x: float = -32.0                      # :29-32
    lidar_max_x: float = 32.0
    lidar_min_y: float = -32.0
    lidar_max_y: float = 32.0
    lidar_seq_len: int = 1                          # :38
    use_ground_plane: bool = False                  # :35
    max_height_lidar: float = 100.0                 # :24
    pixels_per_meter: float = 4.0                   # :25
    hist_max_per_pixel: int = 5                     # :26
    lidar_split_height: float = 0.2                 # :34

    camera_width: int = 1024                        # :40-41
    camera_height: int = 256
    lidar_resolution_width: int = 256               # :42-43
    lidar_resolution_height: int = 256

    img_vert_anchors: int = 256 // 32               # :45-48
    img_horz_anchors: int = 1024 // 32
    lidar_vert_anchors: int = 256 // 32
    lidar_horz_anchors: int = 256 // 32

    block_exp: int = 4                              # :50-53
    n_layer: int = 2
    n_head: int = 4

    tf_d_model: int = 256                           # :73-77
    tf_d_ffn: int = 1024
    tf_num_layers: int = 3
    tf_num_head: int = 8
    tf_dropout: float = 0.0
    num_bounding_boxes: int = 30                    # :80

    # training-loss weights (:82-89) and the agent-loss option (:22-23)
    trajectory_weight: float = 12.0
    trajectory_cls_weight: float = 10.0
    trajectory_reg_weight: float = 8.0
    diff_loss_weight: float = 20.0
    agent_class_weight: float = 10.0
    agent_box_weight: float = 1.0
    bev_semantic_weight: float = 14.0
    latent: bool = False
    latent_rad_thresh: float = 4 * 3.141592653589793 / 9
    # forward_train's timestep range: torch.randint(0, 50) (transfuser_model_v2.py:533)
    train_timestep_max: int = 50

    num_bev_classes: int = 7                        # :116
    bev_features_channels: int = 64                 # :117
    bev_down_sample_factor: int = 4                 # :118
    bev_upsample_factor: int = 2                    # :119

    # Hot-path constants hard-coded in the reference's forward_test
    # (transfuser_model_v2.py:445,476,581,585,594) and DDIMScheduler (:447-451).
    num_modes: int = 20
    num_diff_layers: int = 2
    denoise_steps: int = 2
    trunc_timestep: int = 8
    step_span: int = 20
    num_train_timesteps: int = 1000

    @property
    def lidar_in_channels(self) -> int:
        return 2 * self.lidar_seq_len if self.use_ground_plane else self.lidar_seq_len


def trunk_channels(arch: str):
    """feature_info num_chs of the timm trunk (stem, layer1..4); transfuser_backbone.py:67-96."""
    if arch == "resnet34":
        return [64, 64, 128, 256, 512]
    if arch == "resnet50":
        return [64, 256, 512, 1024, 2048]
    raise ValueError(f"unsupported trunk {arch!r}")


def trunk_blocks(arch: str):
    """(block type, blocks per stage) of the timm trunk."""
    if arch == "resnet34":
        return "basic", [3, 4, 6, 3]
    if arch == "resnet50":
        return "bottleneck", [3, 4, 6, 3]
    raise ValueError(f"unsupported trunk {arch!r}")
