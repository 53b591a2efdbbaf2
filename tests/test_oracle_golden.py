"""CPU: the oracle (CPU restatement) is pinned against the REFERENCE goldens.

The goldens were produced by the reference model itself (``tests/golden/make_golden.py``).
The oracle must reproduce the final trajectory within the north-star bound and every
intermediate / per-(step, layer) output to fp32 rounding.
"""
import os

import numpy as np
import pytest

from golden_util import compare_tap, golden_files, golden_files_r50, load, tap_names, waypoint_l2


@pytest.fixture(scope="module")
def oracle(seeded_sd):
    from oracle.model import OracleModel
    return OracleModel(seeded_sd)


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_inputs_regenerate(path):
    from diffusiondrive_amd.weights import synthetic_inputs
    g = load(path)
    inp = synthetic_inputs(int(g["batch"]), int(g["seed"]))
    for k in ("camera_feature", "lidar_feature", "status_feature", "noise"):
        a = inp[k].astype(np.float64)
        assert abs(a.sum() - float(g[f"in_{k}_sum"])) <= 1e-9 * max(1.0, float(g[f"in_{k}_abssum"]))
    np.testing.assert_array_equal(inp["noise"], g["noise"])
    np.testing.assert_array_equal(inp["status_feature"], g["status_feature"])


@pytest.fixture(scope="module")
def oracle_r50():
    """Config C4: ResNet-50 image trunk on seeded weights (seed 3), the reference's own C4 goldens."""
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.weights import seeded_state_dict
    from oracle.model import OracleModel
    cfg = TransfuserConfig(image_architecture="resnet50")
    return OracleModel(seeded_state_dict(cfg, 3), cfg)


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_oracle_matches_reference(oracle, path):
    _check_oracle(oracle, path)


@pytest.mark.parametrize("path", golden_files_r50(), ids=os.path.basename)
def test_oracle_resnet50_matches_reference(oracle_r50, path):
    """C4 pinned: the oracle's Bottleneck trunk and the 256/512/1024/2048-channel fusion adapters
    (transfuser_backbone.py:66-93) against the reference run with image_architecture="resnet50"."""
    g = load(path)
    assert str(g["image_architecture"]) == "resnet50" and int(g["weight_seed"]) == 3
    _check_oracle(oracle_r50, path)


def _check_oracle(oracle, path):
    from oracle.model import Taps
    from diffusiondrive_amd.weights import synthetic_inputs
    g = load(path)
    inp = synthetic_inputs(int(g["batch"]), int(g["seed"]), oracle.cfg)
    taps = Taps()
    out = oracle.forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"], taps=taps)
    assert waypoint_l2(out["trajectory"].numpy(), g["trajectory"]) <= 2e-5
    np.testing.assert_allclose(out["trajectory"].numpy()[..., 2], g["trajectory"][..., 2], atol=2e-5)
    np.testing.assert_allclose(out["agent_states"].numpy(), g["agent_states"], atol=5e-4)
    np.testing.assert_allclose(out["agent_labels"].numpy(), g["agent_labels"], atol=2e-5)
    for s in range(2):
        for l in range(2):
            np.testing.assert_allclose(taps[f"reg_s{s}l{l}"].numpy(), g[f"reg_s{s}l{l}"], atol=3e-5)
            np.testing.assert_allclose(taps[f"cls_s{s}l{l}"].numpy(), g[f"cls_s{s}l{l}"], atol=3e-5)
    taps["cross_bev_tokens"] = taps["cross_bev"].flatten(2).permute(0, 2, 1)
    taps["bev_semantic_map"] = out["bev_semantic_map"]
    checked = 0
    for name in tap_names(g):
        if name in taps:
            e, cs = compare_tap(g, name, taps[name].numpy())
            assert e <= 1e-5 and cs <= 1e-6, (name, e, cs)
            checked += 1
    assert checked >= 15


def test_oracle_steps_generalise(oracle):
    """steps=N generalises the hard-coded 2 (C5 ablation); steps=2 must be the reference path."""
    from diffusiondrive_amd.weights import synthetic_inputs
    inp = synthetic_inputs(1, 5)
    a = oracle.forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"], heads=False)
    b = oracle.forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"], steps=2,
                       heads=False)
    c = oracle.forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"], steps=4,
                       heads=False)
    assert np.array_equal(a["trajectory"].numpy(), b["trajectory"].numpy())
    assert c["trajectory"].shape == (1, 8, 3) and np.isfinite(c["trajectory"].numpy()).all()


def test_oracle_vanilla_schedule_ignores_anchors(seeded_sd):
    """C5 vanilla DDIM starts from pure noise: the anchors must not influence the result, while the
    truncated (reference) schedule depends on them."""
    import torch
    from diffusiondrive_amd.weights import synthetic_inputs
    from oracle.model import OracleModel
    inp = synthetic_inputs(1, 5)
    sd2 = dict(seeded_sd)
    sd2["_trajectory_head.plan_anchor"] = seeded_sd["_trajectory_head.plan_anchor"] * 0.5
    args = (inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"])
    a = OracleModel(seeded_sd).forward(*args, steps=3, heads=False, schedule="vanilla")["trajectory"]
    b = OracleModel(sd2).forward(*args, steps=3, heads=False, schedule="vanilla")["trajectory"]
    assert torch.equal(a, b)
    c = OracleModel(sd2).forward(*args, steps=2, heads=False)["trajectory"]
    d = OracleModel(seeded_sd).forward(*args, steps=2, heads=False)["trajectory"]
    assert not torch.equal(c, d)
