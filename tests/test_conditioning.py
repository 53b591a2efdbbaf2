"""CPU: how sensitive the reference computation itself is at the bench workload (B = 64, seed 1234).

The oracle (the CPU restatement pinned to the reference goldens) runs twice, the second time with the camera
input perturbed by one fp32 ulp (2^-24 relative, seeded). The change of agent_states under that perturbation
is the floor any fp32-class implementation can be held to; tests/test_parity_gpu.py's AGENT_TOL is tied to it
(10x), and the north-star trajectory bar (1e-4 waypoint L2) must stay far above the trajectory's own change.
"""
import numpy as np
import pytest
import torch

from test_parity_gpu import AGENT_TOL, WAYPOINT_L2_TOL


@pytest.mark.timeout(300)
def test_agent_head_conditioning_bounds_agent_tol(seeded_sd):
    from diffusiondrive_amd.weights import synthetic_inputs
    from oracle.model import OracleModel
    torch.set_num_threads(8)
    m = OracleModel(seeded_sd)
    inp = synthetic_inputs(64, 1234)
    base = m.forward(inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"])
    rng = np.random.default_rng(0)
    cam = (inp["camera_feature"] * (1 + 2.0**-24 * rng.standard_normal(inp["camera_feature"].shape))).astype(np.float32)
    pert = m.forward(cam, inp["lidar_feature"], inp["status_feature"], inp["noise"])
    d_agent = float(np.abs(pert["agent_states"].numpy() - base["agent_states"].numpy()).max())
    d_traj = float(np.abs(pert["trajectory"].numpy() - base["trajectory"].numpy()).max())
    print(f"one-ulp camera perturbation: agent_states {d_agent:.3e}, trajectory {d_traj:.3e}")
    assert 1e-5 < d_agent, "the agent head is no longer ill-conditioned: tighten AGENT_TOL"
    assert AGENT_TOL <= 20 * d_agent, (AGENT_TOL, d_agent)
    assert d_traj < 0.1 * WAYPOINT_L2_TOL
