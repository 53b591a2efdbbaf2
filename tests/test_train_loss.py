"""Training-mode trajectory head + training loss as a loss evaluator: the oracle's
forward_train / LossComputer / transfuser_loss against goldens produced by the REFERENCE's own forward_train and
transfuser_loss (tests/golden/make_train_golden.py), and the GPU path (dd_forward_train) against both."""
import glob
import os

import numpy as np
import pytest
import torch

from golden_util import load, waypoint_l2

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDENS = sorted(glob.glob(os.path.join(HERE, "golden", "train_b*_s*.npz")))
# relative tolerance per loss term. The agent terms inherit the agent head's conditioning: one fp32 ulp on the
# camera input moves agent_states by 1.6-2.4e-4 (tests/test_conditioning.py), and a summation order does as much,
# so the Hungarian-matched box L1 (a sum of |error| over ~36 valid boxes / n_gt) moves by ~1e-4 relative.
LOSS_TOL = {"loss": 1e-5, "trajectory_loss": 1e-5, "agent_class_loss": 5e-4, "agent_box_loss": 5e-4,
            "bev_semantic_loss": 1e-5}
LOSS_KEYS = tuple(LOSS_TOL)


def _case(path):
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
    g = load(path)
    B, seed = int(g["batch"]), int(g["seed"])
    cfg = TransfuserConfig()
    inp = synthetic_inputs(B, seed, cfg)
    targets = {k[len("target_"):]: g[k] for k in g if k.startswith("target_")}
    return g, cfg, seeded_state_dict(cfg, int(g["weight_seed"])), inp, targets


@pytest.fixture(scope="module")
def oracle_runs():
    from oracle.model import OracleModel, transfuser_loss
    runs = []
    for path in GOLDENS:
        g, cfg, sd, inp, targets = _case(path)
        om = OracleModel(sd, cfg)
        out = om.forward_train(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], g["noise"],
                               g["timesteps"], targets)
        runs.append((path, g, out, transfuser_loss(targets, out, cfg)))
    return runs


def test_train_goldens_exist():
    assert len(GOLDENS) >= 2


def test_train_golden_draws_are_the_reference_draw_order():
    """forward_train draws randint(0, 50, (B,)) then randn(B, 20, 8, 2) (transfuser_model_v2.py:533-534): with the
    seed set right before the forward (eval mode: nothing else consumes the generator) the goldens' recorded draws
    are exactly those two calls."""
    for path in GOLDENS:
        g = load(path)
        torch.manual_seed(int(g["seed"]))
        t = torch.randint(0, 50, (int(g["batch"]),))
        nz = torch.randn(int(g["batch"]), 20, 8, 2)
        assert np.array_equal(t.numpy(), g["timesteps"]) and np.array_equal(nz.numpy(), g["noise"])


def test_oracle_forward_train_matches_reference(oracle_runs):
    for path, g, out, _ in oracle_runs:
        for l in range(2):
            reg, cls = out["poses_reg_list"][l].numpy(), out["poses_cls_list"][l].numpy()
            B = reg.shape[0]
            assert waypoint_l2(reg.reshape(B * 20, 8, 3), g[f"reg_l{l}"].reshape(B * 20, 8, 3)) <= 2e-5, path
            assert np.abs(cls - g[f"cls_l{l}"]).max() <= 2e-5, path
        assert waypoint_l2(out["trajectory"].numpy(), g["trajectory"]) <= 2e-5
        for k in ("trajectory_loss_0", "trajectory_loss_1", "trajectory_loss"):
            v = float(out["trajectory_loss_dict"][k]) if k != "trajectory_loss" else float(out[k])
            assert abs(v - float(g[k])) <= 1e-5 * max(1.0, abs(float(g[k]))), (path, k, v, float(g[k]))


def test_oracle_transfuser_loss_matches_reference(oracle_runs):
    for path, g, out, losses in oracle_runs:
        assert np.abs(out["agent_states"].numpy() - g["agent_states"]).max() <= 2e-4
        for k in LOSS_KEYS:
            v, r = float(losses[k]), float(g[f"loss_{k}"])
            assert abs(v - r) <= LOSS_TOL[k] * max(1.0, abs(r)), (path, k, v, r)


def test_agent_loss_host_matches_reference_on_reference_outputs():
    """diffusiondrive_amd.losses.agent_loss (the product's Hungarian-matched agent loss, CPU like the reference's
    cost.cpu()) on the reference's OWN agent outputs and targets: equal to the reference's agent terms."""
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.losses import agent_loss
    cfg = TransfuserConfig()
    for path in GOLDENS:
        g = load(path)
        targets = {k[len("target_"):]: g[k] for k in g if k.startswith("target_")}
        ac, ab = agent_loss(targets, {"agent_states": g["agent_states"], "agent_labels": g["agent_labels"]}, cfg)
        for k, v in (("agent_class_loss", cfg.agent_class_weight * ac), ("agent_box_loss", cfg.agent_box_weight * ab)):
            r = float(g[f"loss_{k}"])
            assert abs(v - r) <= 1e-5 * max(1.0, abs(r)), (path, k, v, r)


@pytest.mark.gpu
@pytest.mark.parametrize("gemm", ["f16x3", "fp32"])
def test_forward_train_matches_reference_goldens(gemm):
    """dd_forward_train through the C ABI (DiffusionDriveModel.forward_train) on the goldens' inputs, timesteps and
    noise: every layer's poses_reg within the north-star waypoint bar of the reference's forward_train, the cls
    logits, the selected trajectory and the LossComputer losses of both layers and their sum."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    for path in GOLDENS:
        g, cfg, sd, inp, targets = _case(path)
        m = DiffusionDriveModel(cfg, sd, device=0, gemm=gemm)
        try:
            feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
            tg = {"trajectory": torch.from_numpy(targets["trajectory"])}
            for _ in range(2):  # eager (first call of the shape), then the captured graph
                out = m.forward_train(feats, tg, timesteps=torch.from_numpy(g["timesteps"]),
                                      noise=torch.from_numpy(g["noise"]), heads=False)
                torch.cuda.synchronize()
                assert m.numerics_flags() == 0
                B = int(g["batch"])
                for l in range(2):
                    reg = out["poses_reg_list"][l].cpu().numpy()
                    cls = out["poses_cls_list"][l].cpu().numpy()
                    assert waypoint_l2(reg.reshape(B * 20, 8, 3), g[f"reg_l{l}"].reshape(B * 20, 8, 3)) <= 1e-4
                    assert np.abs(cls - g[f"cls_l{l}"]).max() <= 1e-4
                assert waypoint_l2(out["trajectory"].cpu().numpy(), g["trajectory"]) <= 1e-4
                for k in ("trajectory_loss_0", "trajectory_loss_1"):
                    v = float(out["trajectory_loss_dict"][k])
                    assert abs(v - float(g[k])) <= 1e-5 * max(1.0, abs(float(g[k]))), (path, gemm, k, v, float(g[k]))
                assert abs(float(out["trajectory_loss"]) - float(g["trajectory_loss"])) <= 1e-5 * float(g["trajectory_loss"])
        finally:
            m.close()


@pytest.mark.gpu
def test_agent_compute_loss_matches_reference_goldens():
    """The agent surface: agent.train(); forward(features, targets) (forward_train on the GPU) and
    compute_loss -> every term of the reference's transfuser_loss (the BEV cross entropy on the GPU, the
    Hungarian-matched agent terms on the CPU), and the eval-mode fallback (L1 of the trajectory)."""
    from diffusiondrive_amd.agent import DiffusionDriveAgent
    for path in GOLDENS:
        g, cfg, sd, inp, targets = _case(path)
        agent = DiffusionDriveAgent(cfg, device=0)
        agent.load_state_dict(sd)
        feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
        tg = {k: torch.from_numpy(v) for k, v in targets.items()}
        agent.train()
        torch.manual_seed(int(g["seed"]))  # the reference's draw order: randint(0, 50) then randn
        pred = agent.forward(feats, tg)
        assert np.array_equal(pred["timesteps"].numpy(), g["timesteps"])
        losses = agent.compute_loss(feats, tg, pred)
        for k in LOSS_KEYS:
            v, r = float(losses[k]), float(g[f"loss_{k}"])
            # the total inherits every term's allowance (the agent terms' dominate: see LOSS_TOL)
            tol = (sum(LOSS_TOL[t] * abs(float(g[f"loss_{t}"])) for t in LOSS_KEYS if t != "loss")
                   + LOSS_TOL["loss"] * abs(r)) if k == "loss" else LOSS_TOL[k] * max(1.0, abs(r))
            assert abs(v - r) <= tol, (path, k, v, r)
        agent.eval()
        ev = agent.compute_loss(feats, tg, agent.forward(feats, noise=torch.from_numpy(g["noise"])))
        assert np.isfinite(float(ev["loss"])) and float(ev["trajectory_loss"]) > 0


@pytest.mark.gpu
def test_forward_train_chunked_batch_reduces_over_the_whole_batch(seeded_sd):
    """B larger than the library's chunk (DDMI_MAX_CHUNK is read at dd_create; 4 here): the losses are reduced over
    all scenes after the chunks, equal to the oracle's batch means."""
    import os as _os
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import synthetic_inputs, synthetic_targets
    from oracle.model import OracleModel
    cfg = TransfuserConfig()
    B = 10
    inp = synthetic_inputs(B, 99, cfg)
    tg = synthetic_targets(B, 99, cfg)
    t = torch.randint(0, 50, (B,), generator=torch.Generator().manual_seed(3))
    _os.environ["DDMI_MAX_CHUNK"] = "4"
    try:
        m = DiffusionDriveModel(cfg, seeded_sd, device=0, gemm="f16x3")
    finally:
        del _os.environ["DDMI_MAX_CHUNK"]
    try:
        feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
        out = m.forward_train(feats, {"trajectory": torch.from_numpy(tg["trajectory"])}, timesteps=t,
                              noise=torch.from_numpy(inp["noise"]), heads=False)
        ref = OracleModel(seeded_sd, cfg).forward_train(inp["camera_feature"], inp["lidar_feature"],
                                                        inp["status_feature"], inp["noise"], t.numpy(), tg, heads=False)
        for k in ("trajectory_loss_0", "trajectory_loss_1"):
            v, r = float(out["trajectory_loss_dict"][k]), float(ref["trajectory_loss_dict"][k])
            assert abs(v - r) <= 1e-5 * max(1.0, abs(r)), (k, v, r)
    finally:
        m.close()
