"""CPU: host-side logic — state-dict schema vs the reference's, weight blob format, DDIM schedule
constants, and that the C-ABI library loads and exports every symbol include/ddmi.h declares
(no compute calls: there is no GPU here)."""
import json
import os
import re
import struct

import numpy as np
import pytest

from golden_util import GOLDEN_DIR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_schema_matches_reference_state_dict():
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.schema import state_dict_schema
    with open(os.path.join(GOLDEN_DIR, "state_dict_schema.json")) as f:
        ref = [(k, tuple(s)) for k, s in json.load(f)]
    mine = [(k, tuple(s)) for k, s, _ in state_dict_schema(TransfuserConfig())]
    assert mine == ref  # same keys, shapes and registration order (763 tensors)
    assert len(mine) == 763


def test_seeded_weights_deterministic_and_param_count(seeded_sd):
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.weights import seeded_state_dict
    n = sum(int(np.prod(v.shape)) for k, v in seeded_sd.items() if v.dtype.kind == "f"
            and not k.endswith(("running_mean", "running_var")))
    assert n == 60715727  # nn.Parameters of V2TransfuserModel (README.md:79 "60M")
    again = seeded_state_dict(TransfuserConfig(), 0)
    for k in ("_backbone.image_encoder.conv1.weight", "bev_proj.0.weight"):
        assert np.array_equal(again[k], seeded_sd[k])


def test_blob_roundtrip_format(seeded_sd):
    from diffusiondrive_amd.weights import pack_blob
    sd = {"a.weight": np.arange(6, dtype=np.float32).reshape(2, 3), "b": np.ones(5, np.float32),
          "c.num_batches_tracked": np.array(3, np.int64)}
    blob = pack_blob(sd)
    assert blob[:4] == b"DDW1"
    (count,) = struct.unpack_from("<I", blob, 4)
    assert count == 2  # integer buffers are not packed
    off = 8
    (nl,) = struct.unpack_from("<I", blob, off)
    off += 4
    assert blob[off:off + nl] == b"a.weight"


def test_strip_prefix():
    from diffusiondrive_amd.weights import strip_prefix
    sd = {"agent._transfuser_model.bev_proj.0.weight": 1, "_transfuser_model.x": 2, "y": 3}
    assert list(strip_prefix(sd)) == ["bev_proj.0.weight", "x", "y"]


def test_check_state_dict_strict(seeded_sd):
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import check_state_dict
    cfg = TransfuserConfig()
    check_state_dict(seeded_sd, cfg)
    bad = dict(seeded_sd)
    bad.pop("bev_proj.0.weight")
    with pytest.raises(RuntimeError):
        check_state_dict(bad, cfg)
    bad = dict(seeded_sd)
    bad["bev_proj.0.weight"] = np.zeros((3, 3), np.float32)
    with pytest.raises(RuntimeError):
        check_state_dict(bad, cfg)


def test_ddim_schedule_bit_exact():
    """The runtime's alphas_cumprod recipe (runtime.cpp) reproduces torch's float32 schedule."""
    import torch
    betas = torch.linspace(1e-4 ** 0.5, 0.02 ** 0.5, 1000, dtype=torch.float32) ** 2
    ac = torch.cumprod(1 - betas, 0).numpy()
    f, d = np.float32, np.float64
    start, end = f(0.01), f(np.sqrt(0.02))
    step = f((end - start) / f(999))
    acc, mine = 1.0, []
    for i in range(1000):
        lin = f(d(step) * d(f(i)) + d(start)) if i < 500 else f(d(-step) * d(f(999 - i)) + d(end))
        acc *= d(f(f(1) - f(lin * lin)))
        mine.append(f(acc))
    assert np.array_equal(np.array(mine, np.float32), ac)


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "ddmi.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dd_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_header_symbols():
    from diffusiondrive_amd import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"libddmi.so does not export {s}"
        assert s in _lib.EXPORTED, f"{s} is not bound in _lib._SIGS"


def test_abi_errors_without_gpu_work():
    """Argument validation runs before any device work and reports through dd_last_error."""
    import ctypes
    from diffusiondrive_amd import _lib
    lib = _lib.load()
    assert lib.dd_forward(None, None, None, None, None, 1, 2, None, None, None, None) == -1
    assert b"null" in lib.dd_last_error()
    cfg = _lib.DDConfig()
    lib.dd_default_config(ctypes.byref(cfg))
    assert (cfg.cam_h, cfg.cam_w, cfg.num_modes, cfg.num_poses, cfg.trunc_timestep) == (256, 1024, 20, 8, 8)
    h = ctypes.c_void_p()
    bad = b"XXXX\0\0\0\0"
    cfg.abi_version = 999
    assert lib.dd_create(ctypes.byref(cfg), bad, len(bad), 0, ctypes.byref(h)) == -1
    assert b"ABI" in lib.dd_last_error()


def test_model_requires_gpu_loudly():
    """No silent CPU fallback: without a GPU the product path raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from diffusiondrive_amd import _lib
    from diffusiondrive_amd.model import DiffusionDriveModel
    with pytest.raises(_lib.DDMIUnavailable):
        DiffusionDriveModel()


def test_inflight_and_runner_lane_counts_validated_before_gpu_work():
    """Batches-in-flight arguments: lanes < 1 is rejected before any handle is built; dd_set_streams validates its
    handle and count through the ABI."""
    import ctypes
    from diffusiondrive_amd import _lib
    from diffusiondrive_amd.model import InFlightPlanner
    from diffusiondrive_amd.runner import BatchedTrajectoryRunner
    with pytest.raises(ValueError):
        InFlightPlanner(lanes=0)
    with pytest.raises(ValueError):
        InFlightPlanner(models=[])
    with pytest.raises(ValueError):
        BatchedTrajectoryRunner(None, lanes=0)
    lib = _lib.load()
    assert lib.dd_set_streams(None, 1) == -1 and b"null" in lib.dd_last_error()
    assert lib.dd_set_streams(ctypes.c_void_p(0), 2) == -1
