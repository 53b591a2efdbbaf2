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
    their own) against lanes = 1 on the same tokens and noise stream: the same {token: Trajectory} map within the
    two-stream / single-stream rounding difference (value_proj split choice, 1e-5 class); the agent's handle is
    back in two-stream mode afterwards."""
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    agent = DiffusionDriveAgent(TransfuserConfig(), device=0)
    agent.load_state_dict(seeded_sd)
    toks = [f"l{i}" for i in range(7)]
    inputs = {t: make_agent_input(700 + i, n_points=3000 + 200 * i) for i, t in enumerate(toks)}
    torch.manual_seed(33)
    one = BatchedTrajectoryRunner(agent, batch_size=2).run(toks, inputs.__getitem__)
    torch.manual_seed(33)
    runner = BatchedTrajectoryRunner(agent, batch_size=2, lanes=3)
    three = runner.run(toks, inputs.__getitem__)
    assert list(three) == toks and len(runner._clones) == 2
    for t in toks:
        assert np.abs(three[t].poses - one[t].poses).max() <= 1e-5, t
    torch.manual_seed(33)
    again = BatchedTrajectoryRunner(agent, batch_size=2).run(toks, inputs.__getitem__)
    for t in toks:
        assert np.array_equal(again[t].poses, one[t].poses), t
