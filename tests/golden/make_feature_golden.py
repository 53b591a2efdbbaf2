#!/usr/bin/env python3
"""Golden vectors for the LiDAR feature by running the REFERENCE builder (build container only).

Runs ``TransfuserFeatureBuilder._get_lidar_feature`` (navsim/agents/diffusiondrive/
transfuser_features.py:79-138) from /root/reference, imported with the offline stubs of
``refshim`` (cv2 / torchvision / nuplan are absent; the LiDAR function needs only numpy), on seeded
synthetic point clouds that include the edge cases of the binning: points exactly on the +-32 m
range ends and on interior bin edges, just outside the range, z exactly at the split height and at
the max height, and NaN coordinates. Stores inputs and outputs only (no reference source); rows 3-5 of lidar_pc (intensity, ring,
lidar id) are zero and unread by the builder, so only the (N, 3) xyz points are kept.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_feature_golden.py
Writes tests/golden/lidar_feat_s{seed}_g{ground_plane}.npz
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

CASES = [(7, False, 20000), (8, True, 20000)]


def make_points(seed, n):
    r = np.random.default_rng(seed)
    pc = np.zeros((6, n), np.float32)  # NAVSIM lidar_pc rows: x, y, z, intensity, ring, lidar id
    pc[0] = r.uniform(-36, 36, n)
    pc[1] = r.uniform(-36, 36, n)
    pc[2] = r.uniform(-1.0, 3.0, n)
    # dense clusters so that many pixels exceed hist_max_per_pixel (the clip)
    k = n // 10
    pc[0, :k] = r.normal(5.0, 0.3, k)
    pc[1, :k] = r.normal(-3.0, 0.3, k)
    pc[2, :k] = r.uniform(0.5, 2.0, k)
    edges = np.array([-32.0, 32.0, -31.75, 0.0, 0.25, 31.75, -32.000004, 32.000004, 15.5, -0.0], np.float32)
    m = 0
    for ex in edges:
        for ey in edges:
            pc[0, k + m], pc[1, k + m], pc[2, k + m] = ex, ey, 1.0
            m += 1
    zs = np.array([0.2, np.nextafter(np.float32(0.2), np.float32(1)), np.nextafter(np.float32(0.2), np.float32(0)),
                   100.0, np.nextafter(np.float32(100), np.float32(0)), -5.0, 150.0], np.float32)
    for z in zs:
        pc[0, k + m], pc[1, k + m], pc[2, k + m] = 1.1, 2.2, z
        m += 1
    pc[0, k + m] = np.nan
    pc[1, k + m + 1] = np.nan
    pc[2, k + m + 2] = np.nan
    return pc


def main():
    import refshim
    refshim.install_stub_finder()
    sys.path.insert(0, "/root/reference")
    from navsim.agents.diffusiondrive.transfuser_config import TransfuserConfig
    from navsim.agents.diffusiondrive.transfuser_features import TransfuserFeatureBuilder

    class _L:
        def __init__(self, pc):
            self.lidar_pc = pc

    class _AI:
        def __init__(self, pc):
            self.lidars = [_L(pc)]

    for seed, ground, n in CASES:
        cfg = TransfuserConfig()
        cfg.use_ground_plane = ground
        pc = make_points(seed, n)
        with np.errstate(invalid="ignore"):
            out = TransfuserFeatureBuilder(cfg)._get_lidar_feature(_AI(pc)).numpy()
        path = os.path.join(HERE, f"lidar_feat_s{seed}_g{int(ground)}.npz")
        np.savez_compressed(path, points_xyz=pc[:3].T.copy(), feature=out, ground_plane=np.array(ground))
        print(path, out.shape, out.dtype, float(out.sum()), int((out == 1).sum()))


if __name__ == "__main__":
    main()
