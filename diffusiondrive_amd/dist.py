"""Scene-parallel execution across the GPUs of one node.

Scenes are independent, so a global batch is sharded contiguously over ranks (rank r gets
scenes [r*B/W, (r+1)*B/W)), every rank runs the full hot path on its shard with replicated
weights, and ONE ``all_gather_into_tensor`` (RCCL over xGMI with the ``nccl`` backend; gloo in
CPU tests) assembles the (B, 8, 3) trajectories in global order. The DDIM start noise of the
global batch is drawn once (seeded) and sliced, so the sharded result equals the single-process
result scene for scene. No other collective exists on this path.
"""
from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist


def shard_bounds(batch: int, rank: int, world: int):
    if batch % world:
        raise ValueError(f"global batch {batch} is not divisible by world size {world}")
    per = batch // world
    return rank * per, (rank + 1) * per


def shard(features: Dict[str, torch.Tensor], rank: int, world: int) -> Dict[str, torch.Tensor]:
    b = next(iter(features.values())).shape[0]
    lo, hi = shard_bounds(b, rank, world)
    return {k: v[lo:hi] for k, v in features.items()}


class ScenePlanner:
    """Wraps a per-device forward ``fn(features, noise) -> (b, 8, 3) trajectories``."""

    def __init__(self, fn: Callable[[Dict[str, torch.Tensor], torch.Tensor], torch.Tensor],
                 group: Optional[dist.ProcessGroup] = None):
        self.fn = fn
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0

    def forward_global(self, features: Dict[str, torch.Tensor], noise: torch.Tensor) -> torch.Tensor:
        """features / noise hold the GLOBAL batch (any device); returns the global trajectories."""
        local = shard(dict(features, noise=noise), self.rank, self.world)
        nz = local.pop("noise")
        return self.gather(self.fn(local, nz))

    def gather(self, traj: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return traj
        traj = traj.contiguous()
        out = torch.empty((traj.shape[0] * self.world,) + tuple(traj.shape[1:]), dtype=traj.dtype, device=traj.device)
        dist.all_gather_into_tensor(out, traj, group=self.group)
        return out
