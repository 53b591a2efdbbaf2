"""Host staging of the raw sensors (features.py camera_features / lidar_features: copy threads into the pinned
stage, one H2D copy) for a batch of 64 NAVSIM-sized scenes, at $DDMI_COPY_THREADS copy threads.

    DDMI_COPY_THREADS=16 python tools/micro/c6_copy.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from diffusiondrive_amd.config import TransfuserConfig  # noqa: E402
from diffusiondrive_amd.features import camera_features, lidar_features  # noqa: E402


def main():
    cfg = TransfuserConfig()
    r = np.random.default_rng(0)
    B, NPTS = 64, 100_000
    imgs = r.integers(0, 256, (B, 3, 1080, 1920, 3), dtype=np.uint8)
    pcs = [np.stack([r.uniform(-40, 40, NPTS), r.uniform(-40, 40, NPTS), r.uniform(-1, 3, NPTS)]).astype(np.float32)
           for _ in range(B)]
    cams = [tuple(imgs[b]) for b in range(B)]
    for _ in range(2):
        camera_features(cams, cfg, 0)
        lidar_features(pcs, cfg, 0)
    torch.cuda.synchronize()
    reps = 8
    t0 = time.perf_counter()
    for _ in range(reps):
        camera_features(cams, cfg, 0)
        lidar_features(pcs, cfg, 0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(f"copy threads {os.environ.get('DDMI_COPY_THREADS', 'default')}: {ms:.2f} ms per 64 scenes "
          f"({B / ms * 1e3:.0f} scenes/s of host staging + features)", flush=True)


if __name__ == "__main__":
    main()
