"""The megakernels' inter-workgroup counters (tfdec_mk4 scene barriers) on the GPU.

Round 5 shipped the four-workgroup tf decoder with its scene counters reset by the kernel itself because a
``hipMemsetAsync`` node zeroing them ahead of the kernel broke replays of the two-stream program. Round 6 traced it
(DESIGN.md §4 tfdec_mk4, ``tools/gpu_r6*.sh``, ``profiles/round6_memset_node.md``): the memset node's zeros were not
what the kernel's memory-side atomic arrivals saw (with the kernel's own reset off the counters carried the previous
launch's counts), only with the runtime's graph packet capture on, only for the counters (the same node on a scratch
buffer, or the counters zeroed by a kernel node with agent-scope atomic stores, were clean). These tests pin what the
product now relies on:

* the captured program holds kernel nodes only (no memset / copy node whose writes a kernel must see);
* a counter the launch did not start from zero fails loudly (DD_NUM_SYNC_STATE) instead of letting a wait pass early,
  and clearing the flags re-zeroes the counters, so the next forward is right;
* a launch whose waits gave up (forced, DD_NUM_SYNC_TIMEOUT) leaves the counters sane for the next launch.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SYNC_TIMEOUT, SYNC_STATE = 2, 4


def _inputs(B, seed):
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(B, seed)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    return feats, torch.from_numpy(inp["noise"])


@pytest.mark.parametrize("streams", [1, 2])
def test_captured_program_has_kernel_nodes_only(gpu, seeded_sd, streams):
    """B = 8 runs the four-workgroup tf decoder and the decoder query groups (the counter users); every segment of
    the captured program must consist of kernel nodes (dd_graph_nodes), and replays must stay bit-identical."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    try:
        m.set_streams(streams)
        feats, nz = _inputs(8, 41)
        outs = [m.forward(feats, noise=nz)["trajectory"] for _ in range(4)]  # eager, capture, replays
        info = m.graph_info()
        assert info["programs"] == 1 and info["kernel_nodes"] > 100, info
        assert info["other_nodes"] == 0, info
        assert m.numerics_flags() == 0
        for o in outs[1:]:
            assert torch.equal(o, outs[0])
    finally:
        m.close()


def _counters(m, B):
    """The tf decoder's scene counters [arrivals][B] + [finishes][B] (the tf_sync_cnt workspace buffer)."""
    return m.tap("tf_sync_cnt").view(torch.int32)[: 2 * B].cpu().numpy()


def test_dirty_tf_counters_fail_loudly_and_heal(gpu, seeded_sd, monkeypatch):
    """Eager forwards (the launch reads the diagnostic knobs per dispatch): a launch with the kernel's reset off
    (DDMI_TF_NORESET) leaves its counters at their final counts (9 barriers x 4 arrivals, 4 finishes); the next
    launch must raise DD_NUM_SYNC_STATE, clearing the flags must re-zero the counters, and the forward after that
    must equal the clean one bit for bit."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    B = 4
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    try:
        m.set_graph(False)
        feats, nz = _inputs(B, 42)
        ref = m.forward(feats, noise=nz)["trajectory"].clone()
        assert m.numerics_flags() == 0
        assert not _counters(m, B).any()
        monkeypatch.setenv("DDMI_TF_NORESET", "1")
        a = m.forward(feats, noise=nz)["trajectory"]
        assert m.numerics_flags(clear=False) == 0  # started clean, left dirty
        assert torch.equal(a, ref)
        np.testing.assert_array_equal(_counters(m, B), [36] * B + [4] * B)
        monkeypatch.delenv("DDMI_TF_NORESET")
        m.forward(feats, noise=nz)
        fl = m.numerics_flags(clear=True)  # the clear re-zeroes the counters
        assert fl & SYNC_STATE, fl
        assert not _counters(m, B).any()
        b = m.forward(feats, noise=nz)["trajectory"]
        assert m.numerics_flags() == 0
        assert torch.equal(b, ref)
    finally:
        m.close()


def test_forced_sync_timeout_leaves_counters_sane(gpu, seeded_sd, monkeypatch):
    """Every wait of one launch gives up after one poll (DDMI_TF_SPIN=1): the launch raises DD_NUM_SYNC_TIMEOUT;
    every workgroup still arrives at every barrier and finishes, so the last to finish resets the counters: they must
    read zero with the flags NOT cleared (no host re-zeroing), and the next launch must be right."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    B = 4
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm="f16x3")
    try:
        m.set_graph(False)
        feats, nz = _inputs(B, 43)
        ref = m.forward(feats, noise=nz)["trajectory"].clone()
        assert m.numerics_flags() == 0
        monkeypatch.setenv("DDMI_TF_SPIN", "1")
        m.forward(feats, noise=nz)
        fl = m.numerics_flags(clear=False)
        assert fl & SYNC_TIMEOUT, fl
        assert not _counters(m, B).any()
        monkeypatch.delenv("DDMI_TF_SPIN")
        b = m.forward(feats, noise=nz)["trajectory"]
        assert torch.equal(b, ref)
        m.numerics_flags(clear=True)
    finally:
        m.close()
