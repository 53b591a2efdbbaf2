"""CPU ORACLE for the input side of the boundary - test infrastructure, never the product.

numpy restatement of ``TransfuserFeatureBuilder`` (navsim/agents/diffusiondrive/
transfuser_features.py:25-138), the checker of the GPU feature builder (``features.hip``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s CPU leg may import it.

* LiDAR (transfuser_features.py:79-138): points with z < max_height_lidar, split at
  lidar_split_height, ``np.histogramdd`` over 256x256 bins of [-32, 32] m (H axis = ego x), clipped
  at hist_max_per_pixel, divided by it, float32. PINNED: ``tests/golden/lidar_feat_*.npz`` hold the
  reference function's own outputs (``tests/golden/make_feature_golden.py`` runs
  ``TransfuserFeatureBuilder._get_lidar_feature`` from /root/reference).
* camera (:57-77): l0 / f0 / r0 crops [28:-28, 416:-416] / [28:-28] stitched side by side,
  ``cv2.resize(img, (1024, 256))`` (INTER_LINEAR), ``transforms.ToTensor()`` (HWC uint8 -> CHW
  float / 255). PARITY UNPINNED: cv2 is absent from this image, so the resize is restated from
  OpenCV's published fixed-point INTER_LINEAR (INTER_RESIZE_COEF_BITS = 11): for the NAVSIM
  geometry (4096x1024 -> 1024x256, an exact factor 4) the source position is 4d + 1.5, both taps
  weigh 0.5 (1024 in Q11) in each direction, and the rounded fixed-point result reduces to
  floor((p00 + p01 + p10 + p11 + 2) / 4) over the 2x2 block at rows / columns 4d+1, 4d+2.
* status (:46-53): [driving_command (4), ego_velocity (2), ego_acceleration (2)].
"""
import numpy as np

CROP_TOP = 28      # transfuser_features.py:68-70
CROP_SIDE = 416


def stitch(cam_l0, cam_f0, cam_r0):
    """transfuser_features.py:68-73."""
    return np.concatenate([cam_l0[CROP_TOP:-CROP_TOP, CROP_SIDE:-CROP_SIDE], cam_f0[CROP_TOP:-CROP_TOP],
                           cam_r0[CROP_TOP:-CROP_TOP, CROP_SIDE:-CROP_SIDE]], axis=1)


def resize_linear_u8(img, out_w, out_h):
    """cv2.resize(img, (out_w, out_h)) INTER_LINEAR for uint8 at an exact even integer factor."""
    h, w = img.shape[:2]
    f = h // out_h
    if img.dtype != np.uint8 or h != f * out_h or w != f * out_w or f % 2:
        raise ValueError("restatement covers uint8 images at an exact even integer down-scale only")
    o = f // 2 - 1
    a = img[o::f][:out_h].astype(np.int32)
    b = img[o + 1::f][:out_h].astype(np.int32)
    s = a[:, o::f][:, :out_w] + a[:, o + 1::f][:, :out_w] + b[:, o::f][:, :out_w] + b[:, o + 1::f][:, :out_w]
    return ((s + 2) >> 2).astype(np.uint8)


def camera_feature(cam_l0, cam_f0, cam_r0, out_w=1024, out_h=256):
    """(3, out_h, out_w) float32 = ToTensor(resize(stitch(...))) (transfuser_features.py:57-77)."""
    r = resize_linear_u8(stitch(cam_l0, cam_f0, cam_r0), out_w, out_h)
    return np.ascontiguousarray(r.transpose(2, 0, 1)).astype(np.float32) / np.float32(255.0)


def lidar_feature(points_xyz, max_height=100.0, split_height=0.2, ground_plane=False, lo=-32, hi=32, ppm=4,
                  hist_max=5):
    """(C, 256, 256) float32 (transfuser_features.py:111-138); points_xyz (N, 3) float32."""
    pc = points_xyz[points_xyz[..., 2] < max_height]
    below = pc[pc[..., 2] <= split_height]
    above = pc[pc[..., 2] > split_height]

    def splat(p):
        bins = np.linspace(lo, hi, (hi - lo) * int(ppm) + 1)
        hist = np.histogramdd(p[:, :2], bins=(bins, bins))[0]
        hist[hist > hist_max] = hist_max
        return hist / hist_max

    feats = [splat(below), splat(above)] if ground_plane else [splat(above)]
    return np.stack(feats, axis=0).astype(np.float32)


def status_feature(driving_command, ego_velocity, ego_acceleration):
    """transfuser_features.py:46-53."""
    return np.concatenate([np.asarray(driving_command, np.float32), np.asarray(ego_velocity, np.float32),
                           np.asarray(ego_acceleration, np.float32)])
