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
    """Wraps a per-device forward ``fn(features, noise) -> (b, 8, 3) trajectories``.

    ``rank`` / ``world`` default to the process group's; passing them explicitly (without a process group)
    lets one process play any rank of a larger world through ``forward_shard`` (the single-GPU rehearsal of
    the 8-GPU configuration in tests/test_sharding_gpu.py)."""

    def __init__(self, fn: Callable[[Dict[str, torch.Tensor], torch.Tensor], torch.Tensor],
                 group: Optional[dist.ProcessGroup] = None, rank: Optional[int] = None,
                 world: Optional[int] = None):
        self.fn = fn
        self.group = group
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        if not 0 <= self.rank < self.world:
            raise ValueError(f"rank {self.rank} outside world {self.world}")

    def forward_shard(self, features: Dict[str, torch.Tensor], noise: torch.Tensor) -> torch.Tensor:
        """features / noise hold the GLOBAL batch; runs this rank's contiguous shard, returns its trajectories."""
        local = shard(dict(features, noise=noise), self.rank, self.world)
        nz = local.pop("noise")
        return self.fn(local, nz)

    def forward_global(self, features: Dict[str, torch.Tensor], noise: torch.Tensor) -> torch.Tensor:
        """features / noise hold the GLOBAL batch (any device); returns the global trajectories."""
        return self.gather(self.forward_shard(features, noise))

    def gather(self, traj: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return traj
        if not dist.is_initialized():
            raise RuntimeError("gather over a world > 1 needs an initialised process group")
        traj = traj.contiguous()
        out = torch.empty((traj.shape[0] * self.world,) + tuple(traj.shape[1:]), dtype=traj.dtype, device=traj.device)
        dist.all_gather_into_tensor(out, traj, group=self.group)
        return out
