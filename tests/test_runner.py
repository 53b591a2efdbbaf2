"""Batched evaluation producer (diffusiondrive_amd/runner.py) vs the per-token reference loop."""
import numpy as np
import pytest
import torch

from test_agent import make_agent_input


def test_batched_noise_draw_equals_per_token_draws():
    """One randn(b, 20, 8, 2) == b successive randn(1, 20, 8, 2) (transfuser_model_v2.py:593)."""
    torch.manual_seed(123)
    seq = torch.cat([torch.randn(1, 20, 8, 2) for _ in range(5)])
    torch.manual_seed(123)
    bat = torch.randn(5, 20, 8, 2)
    assert torch.equal(seq, bat)


@pytest.mark.gpu
def test_runner_matches_per_token_compute_trajectory(gpu, seeded_sd):
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    agent = DiffusionDriveAgent(TransfuserConfig(), device=0)
    agent.load_state_dict(seeded_sd)
    inputs = {f"tok{i}": make_agent_input(100 + i, n_points=5000 + 1000 * i) for i in range(5)}

    def load(tok):
        if tok == "bad":
            raise FileNotFoundError("missing sensor blob")
        return inputs[tok]

    tokens = ["tok0", "tok1", "bad", "tok2", "tok3", "tok4"]
    torch.manual_seed(9)
    runner = BatchedTrajectoryRunner(agent, batch_size=2)
    got = runner.run(tokens, load)
    assert set(got) == set(inputs) and [t for t, _ in runner.failed] == ["bad"]
    torch.manual_seed(9)
    for tok in ["tok0", "tok1", "tok2", "tok3", "tok4"]:  # the reference's per-token loop
        ref = agent.compute_trajectory(inputs[tok])
        l2 = float(np.sqrt(((got[tok].poses[:, :2].astype(np.float64) - ref.poses[:, :2]) ** 2).sum()))
        assert got[tok].poses.shape == (8, 3) and l2 <= 1e-4, (tok, l2)


@pytest.mark.gpu
def test_run_distributed_world1_equals_run(gpu, seeded_sd):
    """runner.run_distributed without a process group (world 1): the whole token list on this rank, the same
    {token: Trajectory} map as run() on the same noise stream."""
    import torch.distributed as dist
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    assert not dist.is_initialized()
    agent = DiffusionDriveAgent(TransfuserConfig(), device=0)
    agent.load_state_dict(seeded_sd)
    toks = [f"d{i}" for i in range(5)]
    inputs = {t: make_agent_input(500 + i, n_points=4000 + 300 * i) for i, t in enumerate(toks)}
    torch.manual_seed(21)
    a = BatchedTrajectoryRunner(agent, batch_size=2).run_distributed(toks, inputs.__getitem__)
    torch.manual_seed(21)
    b = BatchedTrajectoryRunner(agent, batch_size=2).run(toks, inputs.__getitem__)
    assert list(a) == toks and set(b) == set(toks)
    for t in toks:
        assert np.array_equal(a[t].poses, b[t].poses), t


@pytest.mark.gpu
def test_runner_matches_oracle_on_same_noise(gpu, seeded_sd):
    """The batched runner (GPU features + batched forward) against the CPU oracle: oracle features
    (oracle/features.py) and the oracle forward on the same per-scene noise the runner drew
    (torch.manual_seed(9); one randn(b, 20, 8, 2) per batch == successive per-token draws)."""
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    from oracle.model import OracleModel
    from test_agent import _oracle_features
    cfg = TransfuserConfig()
    agent = DiffusionDriveAgent(cfg, device=0)
    agent.load_state_dict(seeded_sd)
    toks = [f"t{i}" for i in range(3)]
    inputs = {t: make_agent_input(300 + i, n_points=8000 + 500 * i) for i, t in enumerate(toks)}
    torch.manual_seed(9)
    got = BatchedTrajectoryRunner(agent, batch_size=2).run(toks, inputs.__getitem__)
    torch.manual_seed(9)
    noise = torch.cat([torch.randn(2, 20, 8, 2), torch.randn(1, 20, 8, 2)])  # the runner's two batches
    f = [_oracle_features(inputs[t]) for t in toks]
    cat = {k: torch.stack([x[k] for x in f]).numpy() for k in f[0]}
    ref = OracleModel(seeded_sd).forward(cat["camera_feature"], cat["lidar_feature"], cat["status_feature"],
                                         noise.numpy(), heads=False)["trajectory"].numpy()
    for i, t in enumerate(toks):
        l2 = float(np.sqrt(((got[t].poses[:, :2].astype(np.float64) - ref[i, :, :2]) ** 2).sum()))
        assert l2 <= 1e-4, (t, l2)


@pytest.mark.gpu
def test_runner_lanes_match_one_lane(gpu, seeded_sd):
    """lanes = 3 (three batches in flight: the agent's handle + 2 clones, single-stream forwards on streams of
    their own) against lanes = 1 on the same tokens and noise stream: the same {token: Trajectory} map (1e-5); the
    agent's handle is back in the stream mode the runner found afterwards."""
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    agent = DiffusionDriveAgent(TransfuserConfig(), device=0)
    agent.load_state_dict(seeded_sd)
    found = agent._transfuser_model.stream_count()
    toks = [f"l{i}" for i in range(7)]
    inputs = {t: make_agent_input(700 + i, n_points=3000 + 200 * i) for i, t in enumerate(toks)}
    torch.manual_seed(33)
    one = BatchedTrajectoryRunner(agent, batch_size=2).run(toks, inputs.__getitem__)
    torch.manual_seed(33)
    runner = BatchedTrajectoryRunner(agent, batch_size=2, lanes=3)
    three = runner.run(toks, inputs.__getitem__)
    assert list(three) == toks and len(runner._clones) == 2
    assert agent._transfuser_model.stream_count() == found  # restored to what the runner found
    for t in toks:
        assert np.abs(three[t].poses - one[t].poses).max() <= 1e-5, t
    runner.close()
    assert runner._clones == []
    # a handle the caller configured two-stream (opt-in) is two-stream again after the lanes
    agent._transfuser_model.set_streams(2)
    torch.manual_seed(33)
    BatchedTrajectoryRunner(agent, batch_size=2, lanes=2).run(toks[:3], inputs.__getitem__)
    assert agent._transfuser_model.stream_count() == 2
    agent._transfuser_model.set_streams(found)
    torch.manual_seed(33)
    again = BatchedTrajectoryRunner(agent, batch_size=2).run(toks, inputs.__getitem__)
    for t in toks:
        assert np.array_equal(again[t].poses, one[t].poses), t


def test_runner_isolates_failures_per_batch(monkeypatch):
    """A failure while building one batch's features, launching its forward or finishing it marks THAT batch's
    tokens failed and the other batches complete (the reference isolates per token: run_pdm_score.py:77-100).
    CPU: stand-in agent / model / feature builder (the isolation logic only; the GPU path is covered above)."""
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner

    class _Stream:
        def synchronize(self):
            pass

    class _Poison:  # a forward output that fails when the batch is finished
        def cpu(self):
            raise RuntimeError("device lost while reading back")

    class _Model:
        device = 0

        def __init__(self):
            self.streams = 2

        def stream_count(self):
            return self.streams

        def set_streams(self, n):
            self.streams = n

        def numerics_flags(self, clear=True):
            return 0

        def forward(self, feats, noise=None, safe=False, stream=None):
            tags = feats["tags"]
            if "boom" in tags:
                raise RuntimeError("forward launch failed")
            if "poison" in tags:
                return {"trajectory": _Poison()}
            return {"trajectory": torch.stack([torch.full((8, 3), float(t[1:])) for t in tags])}

    class _Builder:
        def compute_features_batch(self, inputs):
            if "badfeat" in inputs:
                raise ValueError("corrupt sensor blob")
            return {"tags": list(inputs)}

    class _Agent:
        _config = TransfuserConfig()
        _transfuser_model = _Model()

    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _Stream())
    runner = BatchedTrajectoryRunner.__new__(BatchedTrajectoryRunner)
    runner.agent, runner.batch_size, runner.lanes, runner._clones = _Agent(), 2, 1, []
    runner.device, runner.builder, runner.failed = 0, _Builder(), []
    inputs = {"t0": "t0", "t1": "t1", "t2": "badfeat", "t3": "t3", "t4": "boom", "t5": "t5",
              "t6": "poison", "t7": "t7", "t8": "t8", "t9": "t9"}
    got = runner.run(list(inputs), inputs.__getitem__)
    failed = sorted(t for t, _ in runner.failed)
    assert failed == ["t2", "t3", "t4", "t5", "t6", "t7"], runner.failed
    assert sorted(got) == ["t0", "t1", "t8", "t9"]
    assert float(got["t9"].poses[0, 0]) == 9.0
    assert _Agent._transfuser_model.streams == 2  # untouched with one lane


def test_runner_failed_launch_keeps_lanes_and_pending_aligned(monkeypatch):
    """lanes = 2 and a batch whose forward launch raises: the lane pointer must not advance, so the next batch takes
    the free lane and a lane never holds two pending forwards. Otherwise finishing the older forward would read and
    clear the numerics flag of the newer one on the same lane, and an f16x3 overflow in the newer batch would come
    back unflagged (never re-run in fp32). CPU: stand-in handles whose flag word is per lane."""
    import contextlib

    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner

    class _Stream:
        def __init__(self, *a, **k):
            pass

        def synchronize(self):
            pass

        def wait_stream(self, other):
            pass

    reruns = []

    class _Model:
        device = 0

        def __init__(self):
            self.streams, self.flag, self.busy = 2, 0, 0

        def clone(self):
            return _Model()

        def stream_count(self):
            return self.streams

        def set_streams(self, n):
            self.streams = n

        def numerics_flags(self, clear=True):
            f = self.flag
            if clear:
                self.flag, self.busy = 0, 0
            return f

        def forward(self, feats, noise=None, safe=False, stream=None):
            tags = feats["tags"]
            if "boom" in tags:
                raise RuntimeError("forward launch failed")
            assert self.busy == 0, "a lane took a second batch while its first was still pending"
            self.busy = 1
            if any(t.startswith("ovf") for t in tags):
                self.flag = 1  # this forward overflowed in f16x3
            return {"trajectory": torch.stack([torch.full((8, 3), float(t.lstrip("ovft"))) for t in tags])}

        def rerun_fp32(self, feats, noise, *a, **k):
            reruns.append(tuple(feats["tags"]))
            return {"trajectory": torch.full((len(feats["tags"]), 8, 3), -1.0)}

        def close(self):
            pass

    class _Builder:
        def compute_features_batch(self, inputs):
            return {"tags": list(inputs)}

    class _Agent:
        _config = TransfuserConfig()
        _transfuser_model = _Model()

    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _Stream())
    monkeypatch.setattr(torch.cuda, "Stream", _Stream)
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    runner = BatchedTrajectoryRunner.__new__(BatchedTrajectoryRunner)
    runner.agent, runner.batch_size, runner.lanes, runner._clones = _Agent(), 1, 2, []
    runner.device, runner.builder, runner.failed = 0, _Builder(), []
    toks = ["t0", "boom", "ovf2", "t3", "t4", "boom", "t6", "ovf7"]
    got = runner.run(toks, lambda t: t)
    assert sorted(t for t, _ in runner.failed) == ["boom", "boom"]
    assert sorted(reruns) == [("ovf2",), ("ovf7",)], reruns
    assert float(got["ovf2"].poses[0, 0]) == -1.0 and float(got["ovf7"].poses[0, 0]) == -1.0
    assert float(got["t3"].poses[0, 0]) == 3.0 and float(got["t0"].poses[0, 0]) == 0.0
    assert _Agent._transfuser_model.streams == 2  # restored after the lanes ran single-stream
