"""NAVSIM agent surface of the MI355X DiffusionDrive hot path (the drop-in boundary).

Mirrors ``TransfuserAgent`` (navsim/agents/diffusiondrive/transfuser_agent.py:35-211) and the
``AbstractAgent`` plugin interface (navsim/agents/abstract_agent.py:10-115) for inference:
same constructor signature (Hydra ``_target_`` instantiation, diffusiondrive_agent.yaml:1-17),
``name()``, ``initialize()`` (strict load of ``torch.load(ckpt)['state_dict']`` with ``agent.``
stripped), ``get_sensor_config()``, ``get_feature_builders()``, ``forward(features)`` and
``compute_trajectory(agent_input)``. The forward runs in ``libddmi.so`` on the GPU.

When the real ``navsim`` package is importable the class subclasses its ``AbstractAgent`` and
returns its ``Trajectory`` / ``SensorConfig``; otherwise it uses the local stand-ins below (the GPU
box has no navsim). Training: ``forward`` in training mode runs the trajectory head's forward_train and
``compute_loss`` the reference's transfuser_loss (a loss evaluator over the inference arithmetic: no backward, no
batch-statistics BatchNorm, no dropout); optimizers and target builders are out of scope.
"""
from abc import ABC
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .config import TransfuserConfig, TrajectorySampling
from .features import TransfuserFeatureBuilder
from .model import DiffusionDriveModel

try:  # pragma: no cover - navsim is not installed in this image
    from navsim.agents.abstract_agent import AbstractAgent as _NavsimAbstractAgent
    from navsim.common.dataclasses import SensorConfig as _NavsimSensorConfig
    from navsim.common.dataclasses import Trajectory as _NavsimTrajectory
    HAVE_NAVSIM = True
except Exception:  # noqa: BLE001
    _NavsimAbstractAgent = None
    HAVE_NAVSIM = False


@dataclass
class Trajectory:
    """Stand-in for navsim.common.dataclasses.Trajectory (dataclasses.py:236-248)."""
    poses: np.ndarray
    trajectory_sampling: TrajectorySampling = field(default_factory=TrajectorySampling)

    def __post_init__(self):
        assert self.poses.ndim == 2, "Trajectory poses should have two dimensions for samples and poses."
        assert self.poses.shape[0] == self.trajectory_sampling.num_poses, \
            "Trajectory poses and sampling have unequal number of poses."
        assert self.poses.shape[1] == 3, "Trajectory requires (x, y, heading) at last dim."


@dataclass
class SensorConfig:
    """Stand-in for navsim SensorConfig.build_all_sensors(include=[3]) (transfuser_agent.py:108-110)."""
    include: List[int] = field(default_factory=lambda: [3])
    cam_f0: Any = True
    cam_l0: Any = True
    cam_r0: Any = True
    lidar_pc: Any = True


if HAVE_NAVSIM:  # pragma: no cover
    _Base = _NavsimAbstractAgent
else:
    class _Base(torch.nn.Module, ABC):
        """Local mirror of navsim AbstractAgent (abstract_agent.py:10-115), inference part."""

        def __init__(self, requires_scene: bool = False):
            super().__init__()
            self.requires_scene = requires_scene

        def compute_trajectory(self, agent_input) -> Trajectory:
            """abstract_agent.py:65-86: build features, add batch dim, no-grad forward, Trajectory."""
            self.eval()
            features: Dict[str, torch.Tensor] = {}
            for builder in self.get_feature_builders():
                features.update(builder.compute_features(agent_input))
            features = {k: v.unsqueeze(0) for k, v in features.items()}
            with torch.no_grad():
                predictions = self.forward(features)
                poses = predictions["trajectory"].squeeze(0).cpu().numpy()
            return Trajectory(poses)

        def get_target_builders(self):
            raise NotImplementedError("No target builders. Agent does not support training.")

        def compute_loss(self, features, targets, predictions):
            raise NotImplementedError("No loss. Agent does not support training.")

        def get_optimizers(self):
            raise NotImplementedError("No optimizers. Agent does not support training.")

        def get_training_callbacks(self):
            return []


class DiffusionDriveAgent(_Base):
    """MI355X DiffusionDrive agent; constructor and methods as TransfuserAgent (inference)."""

    def __init__(self, config: Optional[TransfuserConfig] = None, lr: float = 0.0,
                 checkpoint_path: Optional[str] = None, device: Optional[int] = None):
        super().__init__()
        self._config = config or TransfuserConfig()
        self._lr = lr
        self._checkpoint_path = checkpoint_path
        self._transfuser_model = DiffusionDriveModel(self._config, device=device)
        if checkpoint_path:
            self.initialize()

    def name(self) -> str:
        return self.__class__.__name__

    def initialize(self) -> None:
        """transfuser_agent.py:94-106: load ``state_dict`` from the checkpoint, strip ``agent.``,
        strict. Checkpoints are read with ``weights_only=True`` (no pickled code is executed)."""
        if not self._checkpoint_path:
            raise ValueError("DiffusionDriveAgent.initialize() needs checkpoint_path")
        ckpt = torch.load(self._checkpoint_path, map_location="cpu", weights_only=True)
        sd = ckpt["state_dict"] if "state_dict" in ckpt else ckpt
        self.load_state_dict({k.replace("agent.", ""): v for k, v in sd.items()})

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Accepts the reference key schema (``_transfuser_model.``-prefixed or bare model keys)."""
        self._transfuser_model.load_state_dict(state_dict, strict=strict)
        return torch.nn.modules.module._IncompatibleKeys([], [])

    def get_sensor_config(self):
        if HAVE_NAVSIM:  # pragma: no cover
            return _NavsimSensorConfig.build_all_sensors(include=[3])
        return SensorConfig()

    def get_feature_builders(self):
        return [TransfuserFeatureBuilder(config=self._config)]

    def forward(self, features: Dict[str, torch.Tensor], targets: Dict[str, torch.Tensor] = None,
                noise: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        """transfuser_agent.py:120-125. Eval mode: the trajectory plus the auxiliary heads, on the CPU as the
        reference's CPU-feature forward returns them (navsim's compute_trajectory calls ``.numpy()`` on it,
        abstract_agent.py:80-86); numerics-checked (a f16x3 range overflow re-runs the forward in fp32).
        Training mode (``agent.train()``) with targets: the trajectory head's forward_train and its losses
        (transfuser_model_v2.py:502-576) over the network's inference arithmetic - BatchNorm running statistics and
        no dropout (the loss evaluator, dd_forward_train); outputs stay on the device for ``compute_loss``."""
        if self.training and targets is not None:
            return self._transfuser_model.forward_train(features, targets, noise=noise, heads=True)
        out = self._transfuser_model.forward(features, noise=noise, heads=True, safe=True)
        return {k: v.cpu() for k, v in out.items()}

    def compute_loss(self, features: Dict[str, torch.Tensor], targets: Dict[str, torch.Tensor],
                     predictions: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """transfuser_agent.py:127-134 -> transfuser_loss (transfuser_loss.py:11-51): the weighted training loss and
        its terms (diffusiondrive_amd/losses.py). ``predictions`` from ``forward`` in training mode (trajectory
        loss from forward_train) or eval mode (L1 of the trajectory, the reference's fallback)."""
        from .losses import transfuser_loss
        return transfuser_loss(targets, predictions, self._config, self._transfuser_model)

    def forward_trajectory(self, features, noise=None, steps=None) -> Dict[str, torch.Tensor]:
        """Trajectory-only fast path (no BEV-semantic / agent heads)."""
        return self._transfuser_model.forward(features, noise=noise, steps=steps)


# Hydra configs of the reference name the class TransfuserAgent (diffusiondrive_agent.yaml:1-3).
TransfuserAgent = DiffusionDriveAgent
