"""CPU tests of boundary-side logic added for the device noise draw, the chunked forward and the C3 rehearsal:
the Philox restatement against the published known-answer vectors, the global-noise prefix property the C3
test relies on, the rank-injected ScenePlanner, and the bench's CPU-share probe."""
import numpy as np
import pytest
import torch

from philox_ref import device_normals, philox4x32_10


@pytest.mark.parametrize("ctr,key,want", [
    # Random123 kat_vectors, philox4x32 with 10 rounds
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_known_answers(ctr, key, want):
    got = philox4x32_10(np.array([ctr], np.uint32), np.array(key, np.uint32))[0]
    assert [int(v) for v in got] == list(want)


def test_device_normal_restatement_is_standard_normal():
    x = device_normals(1234, 0, 1 << 16).astype(np.float64)
    assert abs(x.mean()) < 0.02 and abs(x.std() - 1) < 0.02
    # a later window of the same stream equals the matching slice of a longer draw
    assert np.array_equal(device_normals(1234, 640, 320), device_normals(1234, 0, 1280)[640:960])


def test_global_noise_prefix_equals_shard0_draw():
    """torch.randn on CPU fills normals in 16-wide blocks; 320 normals per scene keeps the blocks aligned, so
    the first 64 scenes of a 512-scene draw are the 64-scene draw of the same seed (tests/test_sharding_gpu)."""
    from diffusiondrive_amd.weights import reference_noise
    assert np.array_equal(reference_noise(512, 1234)[:64], reference_noise(64, 1234))


def test_scene_planner_rank_injection():
    from diffusiondrive_amd.dist import ScenePlanner
    feats = {"x": torch.arange(16).view(16, 1).float()}
    noise = torch.arange(16).float()
    parts = [ScenePlanner(lambda f, nz: f["x"][:, 0] + 100 * nz, rank=r, world=4).forward_shard(feats, noise)
             for r in range(4)]
    assert torch.equal(torch.cat(parts), feats["x"][:, 0] + 100 * noise)
    with pytest.raises(ValueError):
        ScenePlanner(lambda f, nz: None, rank=4, world=4)
    with pytest.raises(RuntimeError):
        ScenePlanner(lambda f, nz: None, rank=0, world=2).gather(torch.zeros(2, 8, 3))


def test_bench_cpu_share():
    import bench
    share, src = bench.cpu_share()
    assert 1 <= share <= src["sched_getaffinity"]
