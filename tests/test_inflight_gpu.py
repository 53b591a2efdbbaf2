"""Batches in flight (InFlightPlanner, dd_set_streams): several forwards queued at once on one device, each lane a
single-stream captured forward replayed on a stream of its own, must give the results of one forward at a time."""
import numpy as np
import pytest
import torch

from diffusiondrive_amd.config import TransfuserConfig
from diffusiondrive_amd.model import DiffusionDriveModel, InFlightPlanner
from diffusiondrive_amd.weights import synthetic_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KEYS = ("camera_feature", "lidar_feature", "status_feature")


def _inputs(B, seed):
    inp = synthetic_inputs(B, seed, TransfuserConfig())
    return {k: torch.from_numpy(inp[k]).to(DEV) for k in KEYS}, torch.from_numpy(inp["noise"]).to(DEV)


def test_caller_stream_replay_matches_own_stream(gpu_model):
    """A single-stream handle (the default) called on a non-default caller stream replays its graph on that stream
    (no hand-off); called on the default stream it runs on its own stream behind an event hand-off. Same kernels in
    the same order: bit-identical."""
    feats, noise = _inputs(4, 7)
    m = gpu_model
    n0 = m.stream_count()
    try:
        m.set_streams(1)
        ref = m.forward(feats, noise=noise)["trajectory"].cpu()
        s = torch.cuda.Stream(DEV)
        s.wait_stream(torch.cuda.current_stream())
        for _ in range(2):  # eager (first call of the shape), then the captured graph on the caller's stream
            with torch.cuda.stream(s):
                out = m.forward(feats, noise=noise, stream=s)["trajectory"]
            s.synchronize()
            assert torch.equal(out.cpu(), ref)
        # the flag / tap readers wait for a forward that ran on the caller's stream
        assert m.numerics_flags() == 0
        assert m.tap("trajectory").numel() >= 4 * 8 * 3
        assert torch.equal(m.forward(feats, noise=noise)["trajectory"].cpu(), ref)
    finally:
        m.set_streams(n0)


def test_two_stream_graphs_in_a_fresh_process():
    """Two-stream forwards (the default: single-stream graph segments on two streams joined by events) in a child
    process of their own: against the single-stream graph (within 1e-5: the same kernels, another order), the
    training forward's per-layer poses and losses too, and after 8 clones in both modes came and went (DESIGN.md
    section 4, Handle lifetime)."""
    import os
    import subprocess
    import sys
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "two_stream_child.py")
    r = subprocess.run([sys.executable, child], capture_output=True, text=True, timeout=400)
    assert r.returncode == 0 and "two_stream_child: ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])


def test_default_handle_has_no_multi_stream_exec(seeded_sd):
    """The default handle is two-stream, and what it replays is a program of single-stream graph segments: after
    the eager first call and the captured second one, one program of more than one segment, none with parallel
    branches (dd_graph_info counts the root nodes of every segment's graph before instantiation)."""
    m = DiffusionDriveModel(state_dict=seeded_sd, device=0)
    try:
        assert m.stream_count() == 2
        f, nz = _inputs(2, 9)
        outs = [m.forward(f, noise=nz)["trajectory"].cpu() for _ in range(3)]
        info = m.graph_info()
        assert info["programs"] == 1 and info["segments"] > 4 and info["multi_stream_execs"] == 0, info
        assert torch.equal(outs[1], outs[2])  # replays are deterministic
        m.set_streams(1)
        one = m.forward(f, noise=nz)["trajectory"].cpu()
        assert float((one - outs[2]).abs().max()) <= 1e-5
        m.forward(f, noise=nz)
        info = m.graph_info()
        assert {k: info[k] for k in ("programs", "segments", "multi_stream_execs", "other_nodes")} == \
            {"programs": 1, "segments": 1, "multi_stream_execs": 0, "other_nodes": 0}, info
    finally:
        m.close()


@pytest.mark.parametrize("lanes", [2, 3])
def test_inflight_planner_matches_one_at_a_time(seeded_sd, lanes):
    """2 x lanes forwards of different batches queued back to back over the lanes, read after one synchronize:
    every result bit-equal to the same batch run alone on a single-stream handle (the lanes are such handles)."""
    pl = InFlightPlanner(state_dict=seeded_sd, device=0, lanes=lanes)
    solo = DiffusionDriveModel(state_dict=seeded_sd, device=0)
    try:
        batches = [_inputs(4, 100 + i) for i in range(2 * lanes)]
        outs = [pl.forward(f, noise=nz)["trajectory"] for f, nz in batches]
        pl.synchronize()
        assert pl.numerics_flags() == 0
        ref1 = [solo.forward(f, noise=nz)["trajectory"].cpu() for f, nz in batches]
        for i, o in enumerate(outs):
            assert torch.equal(o.cpu(), ref1[i]), f"batch {i} (lane {i % lanes})"
        # distinct batches gave distinct trajectories (no lane read another lane's buffers)
        assert len({float(o.sum()) for o in outs}) == len(outs)
    finally:
        pl.close()
        solo.close()


def test_inflight_planner_one_lane_is_the_plain_handle(seeded_sd):
    pl = InFlightPlanner(state_dict=seeded_sd, device=0, lanes=1)
    solo = DiffusionDriveModel(state_dict=seeded_sd, device=0)
    try:
        f, nz = _inputs(2, 5)
        a = pl.forward(f, noise=nz)["trajectory"].cpu()
        b = solo.forward(f, noise=nz)["trajectory"].cpu()
        assert torch.equal(a, b)
        assert pl.streams == [None]
    finally:
        pl.close()
        solo.close()


def test_set_streams_rejects_bad_count(gpu_model):
    from diffusiondrive_amd import _lib
    with pytest.raises(_lib.DDMIError):
        gpu_model.set_streams(3)
    assert np.isfinite(gpu_model.forward(*_inputs(1, 3)[:1], noise=_inputs(1, 3)[1])["trajectory"].cpu().numpy()).all()


@pytest.mark.parametrize("gemm", ["fp32", "bf16"])
def test_inflight_lanes_in_other_gemm_modes(seeded_sd, gemm):
    """The lanes in the fp32 and bf16 gemm modes (other kernel families on the caller's stream): each batch equals a
    single-stream handle of the same mode bit for bit."""
    pl = InFlightPlanner(state_dict=seeded_sd, device=0, lanes=2, gemm=gemm)
    solo = DiffusionDriveModel(state_dict=seeded_sd, device=0, gemm=gemm)
    try:
        solo.set_streams(1)
        batches = [_inputs(2, 200 + i) for i in range(4)]
        outs = [pl.forward(f, noise=nz)["trajectory"] for f, nz in batches]
        pl.synchronize()
        for i, (f, nz) in enumerate(batches):
            assert torch.equal(outs[i].cpu(), solo.forward(f, noise=nz)["trajectory"].cpu()), (gemm, i)
    finally:
        pl.close()
        solo.close()


def test_inflight_inputs_dropped_right_after_forward(seeded_sd):
    """The lanes read the caller's camera / LiDAR planes in place during the replay. A caller that drops its input
    tensors right after pl.forward() returns and allocates on its own (default) stream must not get that memory
    while a lane still reads it (model.py records the lane stream on the inputs): overwritten inputs would change the
    trajectories."""
    pl = InFlightPlanner(state_dict=seeded_sd, device=0, lanes=2)
    solo = DiffusionDriveModel(state_dict=seeded_sd, device=0)
    try:
        solo.set_streams(1)
        seeds = [300 + i for i in range(6)]
        ref = []
        for sd_ in seeds:
            f, nz = _inputs(8, sd_)
            ref.append(solo.forward(f, noise=nz)["trajectory"].cpu())
        for _ in range(2):  # eager + capture per lane before the timed-like replays
            f, nz = _inputs(8, seeds[0])
            pl.forward(f, noise=nz)
        pl.synchronize()
        outs, junk = [], []
        for sd_ in seeds:
            f, nz = _inputs(8, sd_)
            outs.append(pl.forward(f, noise=nz)["trajectory"])
            shapes = [(v.shape, v.dtype) for v in f.values()] + [(nz.shape, nz.dtype)]
            del f, nz
            # same sizes on the default stream: the caching allocator's first candidates are the dropped blocks
            junk.append([torch.full(sh, float("nan"), dtype=dt, device=DEV) for sh, dt in shapes])
        pl.synchronize()
        for i, o in enumerate(outs):
            assert torch.equal(o.cpu(), ref[i]), f"batch {i}"
    finally:
        pl.close()
        solo.close()


def test_handle_churn_then_replay(seeded_sd):
    """Handle churn (Handle lifetime): 12 clones are created, run (eager, captured, replayed;
    every other one on a caller stream, the rest on their own streams) and destroyed, then the first handle's graph is
    replayed and must give its earlier result bit for bit."""
    base = DiffusionDriveModel(state_dict=seeded_sd, device=0)
    try:
        f, nz = _inputs(1, 41)
        ref = [base.forward(f, noise=nz)["trajectory"].cpu() for _ in range(3)][-1]
        streams = [torch.cuda.Stream(DEV) for _ in range(3)]
        for i in range(12):
            c = base.clone()
            try:
                s = streams[i % 3] if i % 2 else None
                for _ in range(3):
                    if s is not None:
                        s.wait_stream(torch.cuda.current_stream())
                        with torch.cuda.stream(s):
                            out = c.forward(f, noise=nz, stream=s)["trajectory"]
                        s.synchronize()
                    else:
                        out = c.forward(f, noise=nz)["trajectory"]
                assert torch.equal(out.cpu(), ref), i
            finally:
                c.close()
        for _ in range(3):
            again = base.forward(f, noise=nz)["trajectory"].cpu()
        assert torch.equal(again, ref)
    finally:
        base.close()
