"""The C-ABI contract of dd_forward (include/ddmi.h) on the GPU: the nullable noise pointer (device draw), any
batch size (chunked forwards), and the fp32 re-run of a forward that raised the f16x3 numerics flag."""
import ctypes

import numpy as np
import pytest
import torch

from golden_util import waypoint_l2
from philox_ref import device_normals

pytestmark = pytest.mark.gpu
KEYS = ("camera_feature", "lidar_feature", "status_feature")


def _dev_inputs(B, seed):
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(B, seed)
    return {k: torch.from_numpy(inp[k]).cuda() for k in KEYS}, torch.from_numpy(inp["noise"]).cuda()


def test_null_noise_is_the_seeded_device_draw(gpu_model):
    """dd_forward(noise = NULL) through the raw C ABI: the handle draws the Philox / Box-Muller stream of its seed
    (scene s of the stream -> draws [320 s, 320 (s + 1))), equal to the test-side restatement within float32
    libm ulps; the same forward given that noise explicitly is bit-identical; re-seeding repeats the stream."""
    lib = gpu_model.lib
    f, _ = _dev_inputs(3, 17)
    traj = torch.empty(3, 8, 3, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    gpu_model.set_gemm_mode("f16x3")

    def call(noise_ptr):
        rc = lib.dd_forward(gpu_model.handle, f["camera_feature"].data_ptr(), f["lidar_feature"].data_ptr(),
                            f["status_feature"].data_ptr(), noise_ptr, 3, 2, traj.data_ptr(), None, None, s)
        assert rc == 0, lib.dd_last_error()
        torch.cuda.synchronize()
        return traj.clone()

    gpu_model.set_seed(99)
    a = call(None)
    nz_a = gpu_model.tap("in_noise", (3, 20, 8, 2)).clone()
    b = call(None)  # scenes 3..5 of the stream
    nz_b = gpu_model.tap("in_noise", (3, 20, 8, 2)).clone()
    ref = device_normals(99, 0, 6 * 320)
    np.testing.assert_allclose(nz_a.cpu().numpy().reshape(-1), ref[:960], rtol=0, atol=2e-6)
    np.testing.assert_allclose(nz_b.cpu().numpy().reshape(-1), ref[960:], rtol=0, atol=2e-6)
    assert torch.isfinite(a).all() and not torch.equal(a, b)
    assert torch.equal(call(ctypes.c_void_p(nz_a.data_ptr())), a)
    gpu_model.set_seed(99)
    assert torch.equal(call(None), a)
    # through the Python mirror
    gpu_model.set_seed(99)
    assert torch.equal(gpu_model.forward(f, noise="device")["trajectory"], a)
    with pytest.raises(ValueError):
        gpu_model.forward(f, noise="device", safe=True)


def test_null_noise_stream_is_chunk_invariant(seeded_sd, monkeypatch):
    """A device-noise forward of 6 scenes run as chunks of 4 + 2 (DDMI_MAX_CHUNK=4) equals the unchunked one: the
    draw is indexed by scene, not by launch."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    f, _ = _dev_inputs(6, 23)
    outs = []
    for chunk in ("128", "4"):
        monkeypatch.setenv("DDMI_MAX_CHUNK", chunk)
        m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="fp32")
        m.set_seed(5)
        outs.append(m.forward(f, noise="device")["trajectory"].cpu().numpy())
        m.close()
    assert waypoint_l2(outs[0], outs[1]) <= 1e-5


def test_null_noise_shard_equals_unsharded_slice(gpu_model):
    """dd_set_seed_at: a scene shard whose device-noise stream starts at its global scene index draws exactly the
    unsharded run's noise for those scenes (the noise tap is compared bit for bit), so the shard's trajectories
    equal the unsharded run's slice (bit-exact where the kernel routes of B = 6 and B = 3 coincide; 1e-5 bar)."""
    f, _ = _dev_inputs(6, 23)
    gpu_model.set_seed(41)
    full = gpu_model.forward(f, noise="device")["trajectory"].clone()
    nz_full = gpu_model.tap("in_noise", (6, 20, 8, 2)).clone()
    gpu_model.set_seed(41, first_scene=3)
    half = gpu_model.forward({k: v[3:] for k, v in f.items()}, noise="device")["trajectory"].clone()
    nz_half = gpu_model.tap("in_noise", (3, 20, 8, 2)).clone()
    assert torch.equal(nz_half, nz_full[3:])
    assert waypoint_l2(half.cpu().numpy(), full[3:].cpu().numpy()) <= 1e-5
    with pytest.raises(ValueError):
        gpu_model.set_seed(41, first_scene=-1)


def test_flagged_forward_reruns_in_fp32(gpu_model):
    """An input far outside the fp16 range raises DD_NUM_F16_OVERFLOW in f16x3; forward(safe=True) and the batched
    runner's _finish re-run it on the fp32 path (a warning, the fp32 result, the flag cleared)."""
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    f, nz = _dev_inputs(2, 29)
    f["camera_feature"] = f["camera_feature"] * 3.0e5
    gpu_model.set_gemm_mode("fp32")
    ref = gpu_model.forward(f, noise=nz)["trajectory"].clone()
    assert gpu_model.numerics_flags() == 0
    gpu_model.set_gemm_mode("f16x3")
    try:
        gpu_model.numerics_flags(clear=True)
        gpu_model.forward(f, noise=nz)
        assert gpu_model.numerics_flags(clear=True) != 0
        with pytest.warns(UserWarning, match="re-running the forward in fp32"):
            out = gpu_model.forward(f, noise=nz, safe=True)["trajectory"]
        assert torch.equal(out, ref)

        class _Agent:  # the runner only needs the model (and the config for its builder)
            _transfuser_model = gpu_model
            from diffusiondrive_amd.config import TransfuserConfig
            _config = TransfuserConfig()
        runner = BatchedTrajectoryRunner.__new__(BatchedTrajectoryRunner)
        runner.agent = _Agent()
        res = gpu_model.forward(f, noise=nz)
        with pytest.warns(UserWarning):
            got = runner._finish((["t0", "t1"], f, nz, res, gpu_model, None))  # (tokens, feats, noise, out, lane, stream)
        assert np.array_equal(np.stack([got["t0"].poses, got["t1"].poses]), ref.cpu().numpy())
        assert gpu_model.numerics_flags() == 0
    finally:
        gpu_model.set_gemm_mode("fp32")
