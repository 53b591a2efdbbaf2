"""Child process of tests/test_inflight_gpu.py::test_two_stream_graphs_in_a_fresh_process (not collected by pytest):
the opt-in two-stream graphs against the single-stream default, then after handle churn in both modes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.model import DiffusionDriveModel  # noqa: E402
from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs  # noqa: E402


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
    for i in range(16):
        c = one.clone()
        c.set_streams(2 if i % 2 == 0 else 1)
        for _ in range(3):
            o = c.forward(feats, noise=nz)["trajectory"].cpu()
        assert float((o - ref).abs().max()) <= 1e-5, i
        c.close()
    two.set_streams(1)  # lowers the launch stream's priority (the raised stream is destroyed) ...
    two.forward(feats, noise=nz)
    two.set_streams(2)  # ... and the next two-stream forward raises it again
    for _ in range(2):
        again = two.forward(feats, noise=nz)["trajectory"].cpu()
    assert torch.equal(again, out)
    two.close()
    one.close()
    print("two_stream_child: ok", flush=True)


if __name__ == "__main__":
    main()
