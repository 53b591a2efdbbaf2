"""Child process of tests/test_inflight_gpu.py::test_two_stream_graphs_in_a_fresh_process (not collected by pytest):
the two-stream default (single-stream graph segments joined by events) against the single-stream graph, the training
forward in both modes, then after handle churn in both modes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs, synthetic_targets  # noqa: E402


def main():
    cfg = TransfuserConfig()
    inp = synthetic_inputs(4, 7, cfg)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"]).cuda()
    one = DiffusionDriveModel(cfg, seeded_state_dict(cfg, 0), device=0, gemm="f16x3")
    one.set_streams(1)  # explicit: the environment may set the default ($DDMI_STREAMS)
    two = one.clone()
    two.set_streams(2)
    assert one.stream_count() == 1 and two.stream_count() == 2
    ref = [one.forward(feats, noise=nz)["trajectory"].cpu() for _ in range(3)][-1]
    for _ in range(3):  # eager, captured (instantiate + first launch), replayed
        out = two.forward(feats, noise=nz)["trajectory"].cpu()
        assert float((out - ref).abs().max()) <= 1e-5, float((out - ref).abs().max())
    assert two.numerics_flags() == 0
    for i in range(8):
        c = one.clone()
        c.set_streams(2 if i % 2 == 0 else 1)
        for _ in range(3):
            o = c.forward(feats, noise=nz)["trajectory"].cpu()
        assert float((o - ref).abs().max()) <= 1e-5, i
        c.close()
    two.set_streams(1)  # the programs are dropped and re-captured with the other topology
    two.forward(feats, noise=nz)
    two.set_streams(2)
    for _ in range(2):
        again = two.forward(feats, noise=nz)["trajectory"].cpu()
    assert torch.equal(again, out)
    assert two.graph_info()["multi_stream_execs"] == 0
    # the training forward (per-scene FiLM and loss partials around fork / join) in both topologies
    tg = {"trajectory": torch.from_numpy(synthetic_targets(4, 5, cfg)["trajectory"]).cuda()}
    tt = torch.tensor([3, 17, 29, 44])
    r1 = [one.forward_train(feats, tg, timesteps=tt, noise=nz) for _ in range(3)][-1]
    r2 = [two.forward_train(feats, tg, timesteps=tt, noise=nz) for _ in range(3)][-1]
    for l in range(2):
        d = float((r1["poses_reg_list"][l] - r2["poses_reg_list"][l]).abs().max())
        assert d <= 1e-5, ("poses_reg", l, d)
    for k in ("trajectory_loss_0", "trajectory_loss_1"):
        a, b = float(r1["trajectory_loss_dict"][k]), float(r2["trajectory_loss_dict"][k])
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (k, a, b)
    two.close()
    one.close()
    print("two_stream_child: ok", flush=True)


if __name__ == "__main__":
    main()
