"""Seeded synthetic weights / inputs and the weight-blob format handed to ``dd_create``.

There is no network here, so neither the released DiffusionDrive ``.pth`` nor timm's
pretrained ResNet can be fetched. Parity therefore runs on seeded synthetic
weights: every state-dict tensor is drawn from its own numpy PCG64 stream keyed by
(seed, crc32(key)), so any subset regenerates bit-identically on any machine.

Blob format ``DDW1`` (little endian), consumed by ``csrc/weights.cpp``::

    char magic[4] = "DDW1"; uint32 count;
    repeat count: uint32 name_len; char name[name_len]; uint32 ndim; int64 dims[ndim];
                  uint32 dtype (0 = f32); pad to 16 B; float data[prod(dims)]; pad to 16 B
"""
import io
import struct
import zlib
from collections import OrderedDict
from typing import Dict, Mapping

import numpy as np

from .config import TransfuserConfig
from .schema import state_dict_schema

PREFIX = "_transfuser_model."


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))


def synthetic_anchors(num_modes=20, num_poses=8, interval=0.5) -> np.ndarray:
    """k-means-like plan anchors (modes, poses, 2) in metres: speeds × curvatures fan."""
    speeds = np.array([0.0, 2.0, 4.5, 7.0, 9.5, 12.0, 14.0, 16.0, 18.0, 20.0])
    curv = np.array([-0.03, 0.03])
    out = np.zeros((num_modes, num_poses, 2), np.float64)
    m = 0
    for v in speeds:
        for c in curv:
            if m >= num_modes:
                break
            s = v * interval * np.arange(1, num_poses + 1)
            c2 = c * (1.0 + v / 20.0)
            out[m, :, 0] = np.sin(c2 * s) / c2
            out[m, :, 1] = (1.0 - np.cos(c2 * s)) / c2
            m += 1
    return out.astype(np.float32)


def seeded_state_dict(cfg: TransfuserConfig, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Deterministic, numerically well-conditioned weights in the reference key schema.

    Conv/Linear weights are fan-in scaled uniform (variance 1/fan_in, ×2 for convs feeding
    ReLU); BN running statistics are randomised so BN folding is exercised; LayerNorm
    affine parameters are perturbed around (1, 0). Keys/shapes: ``schema.state_dict_schema``.
    """
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape, kind in state_dict_schema(cfg):
        r = _rng(seed, key)
        if kind == "conv":
            fan_in = int(np.prod(shape[1:]))
            b = np.sqrt(6.0 / fan_in)
            a = r.uniform(-b, b, shape)
        elif kind == "linear":
            fan_in = shape[1]
            b = np.sqrt(3.0 / fan_in)
            a = r.uniform(-b, b, shape)
        elif kind == "bias":
            a = r.uniform(-0.1, 0.1, shape)
        elif kind == "bn_w":
            a = r.uniform(0.6, 1.0, shape)
        elif kind == "bn_b":
            a = r.uniform(-0.1, 0.1, shape)
        elif kind == "bn_mean":
            a = r.uniform(-0.1, 0.1, shape)
        elif kind == "bn_var":
            a = r.uniform(0.8, 1.6, shape)
        elif kind == "count":
            sd[key] = np.array(0, dtype=np.int64)
            continue
        elif kind == "ln_w":
            a = r.uniform(0.8, 1.2, shape)
        elif kind == "ln_b":
            a = r.uniform(-0.1, 0.1, shape)
        elif kind in ("pos_emb", "embedding"):
            a = r.normal(0.0, 0.5, shape)
        elif kind == "anchor":
            a = synthetic_anchors(shape[0], shape[1], cfg.trajectory_sampling.interval_length)
        else:
            raise ValueError(kind)
        sd[key] = np.ascontiguousarray(a, dtype=np.float32)
    return sd


def synthetic_inputs(batch: int, seed: int = 1234, cfg: TransfuserConfig = None) -> Dict[str, np.ndarray]:
    """Synthetic scene batch: camera randint/255, sparse LiDAR histogram,
    status [one-hot command, v ~ N(5,3), a ~ N(0,1)], plus the DDIM noise tensor."""
    cfg = cfg or TransfuserConfig()
    r = np.random.Generator(np.random.PCG64([seed, 7]))
    cam = (r.integers(0, 256, (batch, 3, cfg.camera_height, cfg.camera_width)) / 255.0).astype(np.float32)
    lid = r.integers(1, 6, (batch, cfg.lidar_in_channels, cfg.lidar_resolution_height,
                            cfg.lidar_resolution_width)) / 5.0
    lid = lid * (r.random(lid.shape) < 0.1)
    cmd = np.eye(4, dtype=np.float32)[r.integers(0, 4, batch)]
    vel = r.normal(5.0, 3.0, (batch, 2))
    acc = r.normal(0.0, 1.0, (batch, 2))
    status = np.concatenate([cmd, vel, acc], axis=1).astype(np.float32)
    return {
        "camera_feature": cam,
        "lidar_feature": lid.astype(np.float32),
        "status_feature": status,
        "noise": reference_noise(batch, seed, cfg),
    }


def synthetic_targets(batch: int, seed: int = 1234, cfg: TransfuserConfig = None) -> Dict[str, np.ndarray]:
    """Synthetic training targets in the reference's target schema (TransfuserTargetBuilder,
    transfuser_features.py:141-387): ``trajectory`` (B, 8, 3) ego poses of a constant-speed / constant-yaw-rate
    drive (x forward, metres; heading, radians), ``agent_states`` (B, 30, 5) boxes [x, y, heading, length, width]
    (BoundingBox2DIndex), ``agent_labels`` (B, 30) validity, ``bev_semantic_map`` (B, 128, 256) class ids in
    [0, 7) (uint8; the loss takes ``.long()``)."""
    cfg = cfg or TransfuserConfig()
    r = np.random.Generator(np.random.PCG64([seed, 11]))
    P, dt = cfg.trajectory_sampling.num_poses, cfg.trajectory_sampling.interval_length
    v = r.uniform(0.0, 15.0, (batch, 1))
    w = r.normal(0.0, 0.12, (batch, 1))
    tt = dt * np.arange(1, P + 1)[None, :]
    head = w * tt
    safe_w = np.where(np.abs(w) < 1e-6, 1e-6, w)
    x = v * np.sin(safe_w * tt) / safe_w
    y = v * (1.0 - np.cos(safe_w * tt)) / safe_w
    traj = np.stack([x, y, head], axis=-1) + r.normal(0.0, 0.2, (batch, P, 3)) * np.array([1.0, 1.0, 0.05])
    n = cfg.num_bounding_boxes
    boxes = np.stack([r.uniform(-32, 32, (batch, n)), r.uniform(-32, 32, (batch, n)),
                      r.uniform(-np.pi, np.pi, (batch, n)), r.uniform(2.0, 6.0, (batch, n)),
                      r.uniform(1.5, 2.5, (batch, n))], axis=-1)
    labels = r.random((batch, n)) < 0.3
    bev = r.integers(0, 7, (batch, cfg.lidar_resolution_height // 2, cfg.lidar_resolution_width)).astype(np.uint8)
    return {"trajectory": traj.astype(np.float32), "agent_states": boxes.astype(np.float32),
            "agent_labels": labels, "bev_semantic_map": bev}


def reference_noise(batch: int, seed: int, cfg: TransfuserConfig = None) -> np.ndarray:
    """The DDIM start noise exactly as the reference draws it on CPU after
    ``torch.manual_seed(seed)``: ``torch.randn(B, 20, 8, 2)`` (transfuser_model_v2.py:593 is
    the only RNG consumer of the eval forward)."""
    import torch
    cfg = cfg or TransfuserConfig()
    g = torch.Generator().manual_seed(seed)
    shape = (batch, cfg.num_modes, cfg.trajectory_sampling.num_poses, 2)
    return torch.randn(shape, generator=g).numpy()


def strip_prefix(sd: Mapping[str, object]) -> "OrderedDict[str, object]":
    """Reference checkpoint keys → model keys (transfuser_agent.py:94-106 strips ``agent.``;
    the agent's own attribute adds ``_transfuser_model.``)."""
    out = OrderedDict()
    for k, v in sd.items():
        k = k.replace("agent.", "", 1) if k.startswith("agent.") else k
        if k.startswith(PREFIX):
            k = k[len(PREFIX):]
        out[k] = v
    return out


def pack_blob(sd: Mapping[str, np.ndarray]) -> bytes:
    """Serialise a (model-keyed) state dict into the DDW1 blob (float tensors only)."""
    buf = io.BytesIO()
    items = [(k, np.asarray(v)) for k, v in sd.items() if np.asarray(v).dtype.kind == "f"]
    buf.write(b"DDW1")
    buf.write(struct.pack("<I", len(items)))
    for k, v in items:
        v = np.ascontiguousarray(v, dtype=np.float32)
        name = k.encode()
        buf.write(struct.pack("<I", len(name)))
        buf.write(name)
        buf.write(struct.pack("<I", v.ndim))
        for d in v.shape:
            buf.write(struct.pack("<q", d))
        buf.write(struct.pack("<I", 0))
        buf.write(b"\0" * (-buf.tell() % 16))
        buf.write(v.tobytes())
        buf.write(b"\0" * (-buf.tell() % 16))
    return buf.getvalue()
