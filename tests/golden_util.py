"""Helpers to read the committed golden fixtures (tests/golden/ref_b*_s*.npz)."""
import glob
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# oracle tap name -> golden tap name (and layout conversion applied to the oracle tensor)
TAP_MAP = {
    "img_l1": "img_l1", "img_l2": "img_l2", "img_l3": "img_l3", "img_l4": "img_l4",
    "lid_l1": "lid_l1", "lid_l2": "lid_l2", "lid_l3": "lid_l3", "lid_l4": "lid_l4",
    "p3": "p3", "bev_feature": "bev_feature", "keyval": "keyval", "query_out": "query_out",
    "gs_s0l0": "gs_s0l0", "gs_s0l1": "gs_s0l1", "gs_s1l0": "gs_s1l0", "gs_s1l1": "gs_s1l1",
}


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN_DIR, "ref_b*_s*.npz")))


def golden_files_r50():
    """Config C4 goldens: the reference run with image_architecture="resnet50" (make_golden.py ``B:seed:r50``)."""
    return sorted(glob.glob(os.path.join(GOLDEN_DIR, "ref_r50_b*_s*.npz")))


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def tap_names(g):
    return sorted({k[len("tap_"):-len("_sum")] for k in g if k.startswith("tap_") and k.endswith("_sum")
                   and not k.endswith("_abssum")})


def compare_tap(g, name, arr):
    """Return (max abs err on the strided sample, relative checksum error) of ``arr`` vs tap ``name``."""
    a = np.asarray(arr, dtype=np.float64).reshape(-1)
    shape = tuple(g[f"tap_{name}_shape"])
    assert a.size == int(np.prod(shape)), (name, a.size, shape)
    stride = int(g[f"tap_{name}_stride"])
    sample = g[f"tap_{name}_sample"].astype(np.float64)
    err = np.abs(a[::stride] - sample).max()
    scale = max(1.0, np.abs(sample).max())
    cs = abs(a.sum() - float(g[f"tap_{name}_sum"])) / max(1.0, float(g[f"tap_{name}_abssum"]))
    return err / scale, cs


def waypoint_l2(pred, ref):
    """Per-scene L2 over the flattened 8x2 xy waypoints, max over the batch."""
    d = np.asarray(pred, np.float64)[..., :2] - np.asarray(ref, np.float64)[..., :2]
    return float(np.sqrt((d.reshape(d.shape[0], -1) ** 2).sum(-1)).max())
