"""World-size-2 gloo test (CPU) of the scene-parallel path: shard -> per-rank forward ->
all_gather must equal the single-process forward on the same global batch and noise."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _worker(rank, world, port, path, result_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from diffusiondrive_amd.dist import ScenePlanner
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
    from oracle.model import OracleModel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sd = seeded_state_dict(__import__("diffusiondrive_amd.config", fromlist=["x"]).TransfuserConfig(), 0)
    om = OracleModel(sd)
    inp = synthetic_inputs(4, 2024)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}

    def fn(f, nz):
        return om.forward(f["camera_feature"], f["lidar_feature"], f["status_feature"], nz, heads=False)["trajectory"]

    out = ScenePlanner(fn).forward_global(feats, torch.from_numpy(inp["noise"]))
    if rank == 0:
        np.save(result_path, out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_equals_single_process(tmp_path):
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
    from diffusiondrive_amd.config import TransfuserConfig
    from oracle.model import OracleModel
    res = str(tmp_path / "out.npy")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(2, port, str(tmp_path), res), nprocs=2, join=True)
    got = np.load(res)
    inp = synthetic_inputs(4, 2024)
    ref = OracleModel(seeded_state_dict(TransfuserConfig(), 0)).forward(
        inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"], heads=False)["trajectory"]
    assert got.shape == (4, 8, 3)
    np.testing.assert_allclose(got, ref.numpy(), atol=1e-5)


def test_shard_bounds():
    from diffusiondrive_amd.dist import shard_bounds
    assert shard_bounds(512, 3, 8) == (192, 256)
    with pytest.raises(ValueError):
        shard_bounds(10, 0, 3)
