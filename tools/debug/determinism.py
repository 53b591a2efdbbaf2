#!/usr/bin/env python3
"""Run-to-run determinism of the f16x3 forward: two forwards of one handle on the same inputs, compared tap by tap
(bit-identical expected). Environment switches are read at handle creation, so each setting gets its own handle.

    python tools/debug/determinism.py [--batch 4] [--env DDMI_TF_GROUPS=1] ...
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

TAPS = ("query_out", "agent_kv0", "agent_kv1", "ego_out0", "ego_out1", "keyval", "p3")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import numpy as np
    import torch
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs
    from diffusiondrive_amd.config import TransfuserConfig
    cfg = TransfuserConfig()
    m = DiffusionDriveModel(state_dict=seeded_state_dict(cfg, 0), device=0, gemm="f16x3")
    inp = synthetic_inputs(a.batch, 43)
    feats = {k: torch.from_numpy(inp[k]) for k in ("camera_feature", "lidar_feature", "status_feature")}
    nz = torch.from_numpy(inp["noise"])
    runs = []
    for _ in range(a.reps):
        out = m.forward(feats, noise=nz)["trajectory"].numpy()
        taps = {}
        for t in TAPS:
            try:
                taps[t] = m.tap(t).cpu().numpy().copy()
            except Exception:  # noqa: BLE001 - a tap this build does not keep
                pass
        runs.append((out, taps, m.numerics_flags(clear=True)))
    o0, t0, f0 = runs[0]
    for i, (o, t, f) in enumerate(runs[1:], 1):
        print(f"[{' '.join(a.env) or 'default'} B={a.batch}] run {i}: flags {f0}/{f} trajectory "
              f"{'identical' if np.array_equal(o, o0) else 'DIFF %.3e' % float(np.abs(o - o0).max())}", flush=True)
        for k in t0:
            if k in t and not np.array_equal(t[k], t0[k]):
                d = np.abs(t[k] - t0[k])
                print(f"   tap {k}: max diff {d.max():.3e} at {np.unravel_index(int(d.argmax()), d.shape)}, "
                      f"{int((d > 0).sum())} elements differ", flush=True)


if __name__ == "__main__":
    main()
