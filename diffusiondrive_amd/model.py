"""Host-side model object over the ddmi C ABI: the MI355X replacement of ``V2TransfuserModel``.

``DiffusionDriveModel.forward(features)`` has the reference's contract
(transfuser_model_v2.py:98-162, eval mode): a feature dict with ``camera_feature``
(B,3,256,1024), ``lidar_feature`` (B,1,256,256), ``status_feature`` (B,8) in, a dict with
``trajectory`` (B,8,3) out (plus ``bev_semantic_map`` / ``agent_states`` / ``agent_labels`` when
``heads=True``). The forward runs entirely in ``libddmi.so`` on the GPU; PyTorch only provides
device memory and the stream. There is no CPU fallback: without the library or a GPU it raises.
"""
import contextlib
import ctypes
import os
import warnings
from typing import Dict, List, Mapping, Optional

import numpy as np
import torch

from . import _lib
from .config import TransfuserConfig
from .schema import state_dict_schema
from .weights import pack_blob, strip_prefix

ARCH_CODE = {"resnet34": 34, "resnet50": 50}


def make_dd_config(cfg: TransfuserConfig) -> _lib.DDConfig:
    c = _lib.DDConfig()
    lib = _lib.load()
    lib.dd_default_config(c)
    c.image_arch = ARCH_CODE[cfg.image_architecture]
    c.lidar_arch = ARCH_CODE[cfg.lidar_architecture]
    c.cam_h, c.cam_w = cfg.camera_height, cfg.camera_width
    c.lidar_h, c.lidar_w = cfg.lidar_resolution_height, cfg.lidar_resolution_width
    c.lidar_channels = cfg.lidar_in_channels
    c.num_modes = cfg.num_modes
    c.num_poses = cfg.trajectory_sampling.num_poses
    c.trunc_timestep = cfg.trunc_timestep
    c.step_span = cfg.step_span
    return c


def check_state_dict(sd: Mapping[str, object], cfg: TransfuserConfig, strict: bool = True):
    """Key / shape check against the reference schema (load_state_dict(strict=True) semantics,
    transfuser_agent.py:94-106). Returns (missing, unexpected); raises on mismatch if strict."""
    schema = {k: tuple(s) for k, s, _ in state_dict_schema(cfg)}
    missing = [k for k in schema if k not in sd]
    unexpected = [k for k in sd if k not in schema]
    bad = [k for k in schema if k in sd and tuple(np.shape(np.asarray(_to_np(sd[k])))) != schema[k]]
    if strict and (missing or unexpected or bad):
        raise RuntimeError(
            f"Error(s) in loading state_dict: missing={missing[:5]}{'...' if len(missing) > 5 else ''} "
            f"unexpected={unexpected[:5]} shape_mismatch={bad[:5]}")
    return missing, unexpected


def _to_np(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return np.asarray(v)


class DiffusionDriveModel:
    """The DiffusionDrive inference forward on one MI355X (one handle per process/device)."""

    def __init__(self, config: Optional[TransfuserConfig] = None, state_dict: Optional[Mapping] = None,
                 device: Optional[int] = None, gemm: Optional[str] = None):
        """``gemm``: conv / linear arithmetic, 'f16x3' (default: fp32-class 3-product fp16 split
        MFMA), 'fp32' (fp32 MFMA) or 'bf16' (reduced precision); $DDMI_GEMM overrides the default."""
        self.config = config or TransfuserConfig()
        self._gemm = gemm or os.environ.get("DDMI_GEMM", "f16x3")
        if self._gemm not in self.GEMM_MODES:
            raise ValueError(f"gemm mode must be one of {sorted(self.GEMM_MODES)}, got {self._gemm!r}")
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.DDMIUnavailable("DiffusionDriveModel needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.cuda.current_device() if device is None else int(device)
        self._h = None
        if state_dict is not None:
            self.load_state_dict(state_dict)

    # ------------------------------------------------------------------ weights
    def load_state_dict(self, state_dict: Mapping, strict: bool = True):
        sd = strip_prefix(state_dict)
        check_state_dict(sd, self.config, strict)
        blob = pack_blob({k: _to_np(v) for k, v in sd.items()})
        cfg = make_dd_config(self.config)
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(blob, len(blob))
        with torch.cuda.device(self.device):
            _lib.check(self.lib.dd_create(ctypes.byref(cfg), ctypes.cast(buf, ctypes.c_void_p), len(blob),
                                          self.device, ctypes.byref(h)), self.lib)
        del buf
        self.close()
        self._h = h
        self._blob = blob  # clone() re-creates a handle from it (batches-in-flight lanes)
        self.set_gemm_mode(self._gemm)
        return self

    def clone(self) -> "DiffusionDriveModel":
        """Another handle on the same device with the same weights, gemm mode and schedule (its own buffers,
        streams and captured graphs): a lane of InFlightPlanner / the batched runner."""
        if getattr(self, "_blob", None) is None:
            raise RuntimeError("DiffusionDriveModel has no weights loaded (call load_state_dict)")
        m = DiffusionDriveModel(self.config, device=self.device, gemm=self.gemm_mode())
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(self._blob, len(self._blob))
        with torch.cuda.device(self.device):
            _lib.check(self.lib.dd_create(ctypes.byref(make_dd_config(self.config)), ctypes.cast(buf, ctypes.c_void_p),
                                          len(self._blob), self.device, ctypes.byref(h)), self.lib)
        m._h, m._blob = h, self._blob
        m.set_gemm_mode(m._gemm)
        if getattr(self, "_schedule", None):
            m.set_schedule(self._schedule)
        return m

    def close(self):
        if self._h is not None and self._h.value:
            self.lib.dd_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("DiffusionDriveModel has no weights loaded (call load_state_dict)")
        return self._h

    # ------------------------------------------------------------------ forward
    def _dev(self, t, dtype=torch.float32):
        t = torch.as_tensor(t)
        return t.to(device=f"cuda:{self.device}", dtype=dtype).contiguous()

    def forward(self, features: Dict[str, torch.Tensor], noise: Optional[torch.Tensor] = None,
                steps: Optional[int] = None, heads: bool = False, modes: bool = False,
                stream: Optional[torch.cuda.Stream] = None, safe: bool = False) -> Dict[str, torch.Tensor]:
        """``noise``: the DDIM start noise (B,20,8,2); None draws it on the CPU as the reference does
        (``torch.randn``, transfuser_model_v2.py:593); ``"device"`` lets the library draw it on the GPU
        (Philox stream of ``set_seed``; N(0,1) but not torch.randn's values).
        ``safe``: synchronise, and if a kernel raised a numerics flag (f16x3 activation beyond
        the fp16 range) re-run this forward in fp32 and warn; never returns a flagged result."""
        if not safe:
            return self._forward(features, noise, steps, heads, modes, stream)
        if isinstance(noise, str):
            raise ValueError("safe=True re-runs a flagged forward on the same noise: pass a tensor (or None)")
        if noise is None:
            B = torch.as_tensor(features["status_feature"]).shape[0]
            noise = torch.randn((B, self.config.num_modes, self.config.trajectory_sampling.num_poses, 2))
        self.numerics_flags(clear=True)
        out = self._forward(features, noise, steps, heads, modes, stream)
        if self.numerics_flags(clear=True):
            out = self.rerun_fp32(features, noise, steps, heads, modes, stream)
        return out

    def rerun_fp32(self, features, noise, steps=None, heads=False, modes=False, stream=None):
        """Re-run a forward whose numerics flag was raised directly on the fp32-MFMA path (warns; raises if
        the fp32 forward raises a flag as well). ``noise`` must be the tensor the flagged forward used."""
        mode = self.gemm_mode()
        warnings.warn(f"ddmi: numerics flag raised in gemm mode {mode!r}; re-running the forward in fp32")
        self.set_gemm_mode("fp32")
        try:
            out = self._forward(features, noise, steps, heads, modes, stream)
        finally:
            self.set_gemm_mode(mode)
        if self.numerics_flags(clear=True):
            raise _lib.DDMIError("numerics flag raised by the fp32 forward as well")
        return out

    def set_seed(self, seed: int, first_scene: int = 0):
        """Seed of the device noise draw (``noise="device"``); restarts its stream at global scene index
        ``first_scene`` (dd_set_seed_at: a scene shard starting at that index draws the unsharded run's noise)."""
        if first_scene < 0:
            raise ValueError("first_scene must be >= 0")
        _lib.check(self.lib.dd_set_seed_at(self.handle, int(seed) & (2 ** 64 - 1), int(first_scene)), self.lib)

    def _forward(self, features, noise, steps, heads, modes, stream) -> Dict[str, torch.Tensor]:
        # stage inputs and allocate outputs on the stream the forward is ordered after, so the caching
        # allocator ties their lifetime to it (the handle's stream waits on that stream and hands back to it)
        dev = torch.device(f"cuda:{self.device}")
        s = stream or torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            return self._forward_on(features, noise, steps, heads, modes, s)

    def _forward_on(self, features, noise, steps, heads, modes, s) -> Dict[str, torch.Tensor]:
        cfg = self.config
        cam = features["camera_feature"]
        out_device = cam.device if isinstance(cam, torch.Tensor) else torch.device("cpu")
        cam = self._dev(cam)
        lid = self._dev(features["lidar_feature"])
        st = self._dev(features["status_feature"])
        B = st.shape[0]
        Q, P = cfg.num_modes, cfg.trajectory_sampling.num_poses
        if tuple(cam.shape) != (B, 3, cfg.camera_height, cfg.camera_width):
            raise ValueError(f"camera_feature must be (B,3,{cfg.camera_height},{cfg.camera_width}), got {tuple(cam.shape)}")
        if tuple(lid.shape) != (B, cfg.lidar_in_channels, cfg.lidar_resolution_height, cfg.lidar_resolution_width):
            raise ValueError(f"lidar_feature has shape {tuple(lid.shape)}")
        if tuple(st.shape) != (B, 8):
            raise ValueError(f"status_feature must be (B,8), got {tuple(st.shape)}")
        if noise is None:
            # the reference draws its DDIM start noise here (transfuser_model_v2.py:593), on CPU
            noise = torch.randn((B, Q, P, 2))
        if isinstance(noise, str):
            if noise != "device":
                raise ValueError(f"noise must be a tensor, None or 'device', got {noise!r}")
            nz = None
        else:
            nz = self._dev(noise)
            if tuple(nz.shape) != (B, Q, P, 2):
                raise ValueError(f"noise must be (B,{Q},{P},2), got {tuple(nz.shape)}")
        # the graph reads the camera / LiDAR planes in place (through the handle's input table) and copies status /
        # noise on stream s: a caller that drops its tensors right after forward() returns must not have their
        # memory handed to other work while s still reads it (tensors allocated on another stream)
        for t in (cam, lid, st, nz):
            if t is not None:
                t.record_stream(s)
        dev = cam.device
        traj = torch.empty((B, P, 3), device=dev)
        outs = _lib.DDOutputs()
        outs.trajectory = traj.data_ptr()
        res = {"trajectory": traj}
        if modes:
            res["poses_reg"] = torch.empty((B, Q, P, 3), device=dev)
            res["poses_cls"] = torch.empty((B, Q), device=dev)
            outs.poses_reg = res["poses_reg"].data_ptr()
            outs.poses_cls = res["poses_cls"].data_ptr()
        if heads:
            res["bev_semantic_map"] = torch.empty(
                (B, 7, cfg.lidar_resolution_height // 2, cfg.lidar_resolution_width), device=dev)
            res["agent_states"] = torch.empty((B, cfg.num_bounding_boxes, 5), device=dev)
            res["agent_labels"] = torch.empty((B, cfg.num_bounding_boxes), device=dev)
            outs.bev_semantic_map = res["bev_semantic_map"].data_ptr()
            outs.agent_states = res["agent_states"].data_ptr()
            outs.agent_labels = res["agent_labels"].data_ptr()
        _lib.check(self.lib.dd_forward_ex(self.handle, cam.data_ptr(), lid.data_ptr(), st.data_ptr(),
                                          nz.data_ptr() if nz is not None else None,
                                          B, int(steps or cfg.denoise_steps), ctypes.byref(outs),
                                          s.cuda_stream), self.lib)
        if out_device.type != "cuda":
            res = {k: v.to(out_device) for k, v in res.items()}
        return res

    __call__ = forward

    def forward_train(self, features: Dict[str, torch.Tensor], targets: Optional[Dict[str, torch.Tensor]] = None,
                      timesteps: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                      heads: bool = True, stream: Optional[torch.cuda.Stream] = None,
                      safe: bool = True) -> Dict[str, torch.Tensor]:
        """V2TransfuserModel.forward(features, targets) with the trajectory head in training mode
        (TrajectoryHead.forward_train, transfuser_model_v2.py:520-576) over the eval-mode network (dropout off,
        BatchNorm running statistics): the deterministic loss evaluator (dd_forward_train).

        ``timesteps`` (B,) and ``noise`` (B, 20, 8, 2) are forward_train's two random draws; None draws them as the
        reference does, in its order, from the global CPU generator (``torch.randint(0, 50, (B,))`` then
        ``torch.randn``, :533-534). Returns ``trajectory`` (the last layer's argmax mode), ``poses_reg_list`` /
        ``poses_cls_list`` (every layer), ``timesteps`` / ``noise`` (the draws used) and, with ``targets``
        (``trajectory`` (B, 8, 3)), ``trajectory_loss`` and ``trajectory_loss_dict`` (LossComputer per layer,
        modules/multimodal_loss.py:119-168) as 0-d tensors; ``heads`` adds the BEV-semantic / agent outputs.
        The outputs are ordered on the current stream when this returns (also with an explicit ``stream``).
        ``safe`` (default): synchronise, and if a kernel raised a numerics flag (f16x3 activation beyond the fp16
        range) re-run the call in fp32 with the same draws and warn, as ``forward(safe=True)`` does."""
        cfg = self.config
        B = torch.as_tensor(features["status_feature"]).shape[0]
        Q, P = cfg.num_modes, cfg.trajectory_sampling.num_poses
        if timesteps is None:
            timesteps = torch.randint(0, cfg.train_timestep_max, (B,))
        if noise is None:
            noise = torch.randn((B, Q, P, 2))
        if not safe:
            return self._forward_train(features, targets, timesteps, noise, heads, stream)
        self.numerics_flags(clear=True)
        res = self._forward_train(features, targets, timesteps, noise, heads, stream)
        if self.numerics_flags(clear=True):
            mode = self.gemm_mode()
            warnings.warn(f"ddmi: numerics flag raised in gemm mode {mode!r}; re-running forward_train in fp32")
            self.set_gemm_mode("fp32")
            try:
                res = self._forward_train(features, targets, timesteps, noise, heads, stream)
            finally:
                self.set_gemm_mode(mode)
            if self.numerics_flags(clear=True):
                raise _lib.DDMIError("numerics flag raised by the fp32 forward_train as well")
        return res

    def _forward_train(self, features, targets, timesteps, noise, heads, stream) -> Dict[str, torch.Tensor]:
        cfg = self.config
        dev = torch.device(f"cuda:{self.device}")
        cur = torch.cuda.current_stream(dev)
        s = stream or cur
        B = torch.as_tensor(features["status_feature"]).shape[0]
        Q, P = cfg.num_modes, cfg.trajectory_sampling.num_poses
        with torch.cuda.stream(s):
            cam = self._dev(features["camera_feature"])
            lid = self._dev(features["lidar_feature"])
            st = self._dev(features["status_feature"])
            nz = self._dev(noise)
            tt = self._dev(timesteps, dtype=torch.int32)
            if tuple(nz.shape) != (B, Q, P, 2) or tuple(tt.shape) != (B,):
                raise ValueError(f"noise must be (B,{Q},{P},2) and timesteps (B,), got {tuple(nz.shape)}, {tuple(tt.shape)}")
            if int(tt.min()) < 0 or int(tt.max()) >= cfg.num_train_timesteps:
                raise ValueError(f"timesteps must lie in [0, {cfg.num_train_timesteps})")
            tg = None
            if targets is not None and targets.get("trajectory") is not None:
                tg = self._dev(targets["trajectory"])
                if tuple(tg.shape) != (B, P, 3):
                    raise ValueError(f"targets['trajectory'] must be (B,{P},3), got {tuple(tg.shape)}")
            for t in (cam, lid, st, nz, tt, tg):
                if t is not None:
                    t.record_stream(s)
            res = {"trajectory": torch.empty((B, P, 3), device=dev),
                   "poses_reg_list": [torch.empty((B, Q, P, 3), device=dev) for _ in range(2)],
                   "poses_cls_list": [torch.empty((B, Q), device=dev) for _ in range(2)]}
            outs = _lib.DDTrainOutputs()
            outs.trajectory = res["trajectory"].data_ptr()
            for l in range(2):
                outs.poses_reg[l] = res["poses_reg_list"][l].data_ptr()
                outs.poses_cls[l] = res["poses_cls_list"][l].data_ptr()
            loss = None
            if tg is not None:
                loss = torch.empty(3, device=dev)
                outs.loss = loss.data_ptr()
            if heads:
                res["bev_semantic_map"] = torch.empty((B, 7, cfg.lidar_resolution_height // 2,
                                                       cfg.lidar_resolution_width), device=dev)
                res["agent_states"] = torch.empty((B, cfg.num_bounding_boxes, 5), device=dev)
                res["agent_labels"] = torch.empty((B, cfg.num_bounding_boxes), device=dev)
                outs.bev_semantic_map = res["bev_semantic_map"].data_ptr()
                outs.agent_states = res["agent_states"].data_ptr()
                outs.agent_labels = res["agent_labels"].data_ptr()
            _lib.check(self.lib.dd_forward_train(self.handle, cam.data_ptr(), lid.data_ptr(), st.data_ptr(),
                                                 nz.data_ptr(), tt.data_ptr(), tg.data_ptr() if tg is not None else None,
                                                 B, float(cfg.trajectory_cls_weight), float(cfg.trajectory_reg_weight),
                                                 ctypes.byref(outs), s.cuda_stream), self.lib)
        if s != cur:
            # the outputs (the loss reduction last) were written on s: order the caller's stream after it, so a
            # .cpu() / .item() on the current stream reads finished values
            cur.wait_stream(s)
            for t in [res["trajectory"], *res["poses_reg_list"], *res["poses_cls_list"], loss,
                      res.get("bev_semantic_map"), res.get("agent_states"), res.get("agent_labels")]:
                if t is not None:
                    t.record_stream(cur)
        res["timesteps"] = torch.as_tensor(timesteps)
        res["noise"] = torch.as_tensor(noise)
        if loss is not None:
            res["trajectory_loss_dict"] = {"trajectory_loss_0": loss[0], "trajectory_loss_1": loss[1]}
            res["trajectory_loss"] = loss[2]
        return res

    # ------------------------------------------------------------------ instrumentation
    def tap(self, name: str, shape=None) -> torch.Tensor:
        """Copy a named internal buffer of the last forward (NHWC device layout) to a tensor."""
        n = ctypes.c_size_t()
        _lib.check(self.lib.dd_tap(self.handle, name.encode(), None, 0, ctypes.byref(n), None), self.lib)
        t = torch.empty(n.value, device=f"cuda:{self.device}")
        _lib.check(self.lib.dd_tap(self.handle, name.encode(), t.data_ptr(), n.value, ctypes.byref(n),
                                   torch.cuda.current_stream(self.device).cuda_stream), self.lib)
        return t if shape is None else t[: int(np.prod(shape))].view(*shape)

    GEMM_MODES = {"fp32": 0, "f16x3": 1, "bf16": 2}

    def set_gemm_mode(self, mode: str):
        """'fp32' (fp32-input MFMA), 'f16x3' (3-product fp16 split MFMA, fp32-class) or 'bf16'
        (one bf16 product per MAC: reduced precision); include/ddmi.h."""
        if mode not in self.GEMM_MODES:
            raise ValueError(f"gemm mode must be one of {sorted(self.GEMM_MODES)}, got {mode!r}")
        _lib.check(self.lib.dd_set_gemm_mode(self.handle, self.GEMM_MODES[mode]), self.lib)

    SCHEDULES = {"truncated": 0, "vanilla": 1}

    def set_schedule(self, schedule: str):
        """'truncated' (the reference's 2-step truncated DDIM) or 'vanilla' (C5 ablation: x_T = noise,
        set_timesteps(steps) over 1000 train steps)."""
        if schedule not in self.SCHEDULES:
            raise ValueError(f"schedule must be one of {sorted(self.SCHEDULES)}, got {schedule!r}")
        _lib.check(self.lib.dd_set_schedule(self.handle, self.SCHEDULES[schedule]), self.lib)
        self._schedule = schedule

    def gemm_mode(self) -> str:
        m = ctypes.c_int()
        _lib.check(self.lib.dd_get_gemm_mode(self.handle, ctypes.byref(m)), self.lib)
        return {v: k for k, v in self.GEMM_MODES.items()}[m.value]

    def numerics_flags(self, clear: bool = True) -> int:
        """DD_NUM_* bits raised since the last clear (bit 0: f16x3 activation overflow)."""
        f = ctypes.c_uint()
        _lib.check(self.lib.dd_numerics_flags(self.handle, ctypes.byref(f), int(clear)), self.lib)
        return f.value

    def set_profiling(self, on: bool):
        _lib.check(self.lib.dd_set_profiling(self.handle, int(on)), self.lib)

    def set_graph(self, on: bool):
        _lib.check(self.lib.dd_set_graph(self.handle, int(on)), self.lib)

    def set_streams(self, n: int):
        """2 (default): the forward runs its independent branches (LiDAR trunk, tf decoder, heads) on a second
        stream; it is captured as single-stream graph segments joined by events between their launches (no
        multi-stream graph exec: DESIGN.md section 4, Handle lifetime). 1: one stream, and a forward called on a
        non-default stream runs on that stream itself (the per-lane mode of InFlightPlanner). dd_set_streams."""
        _lib.check(self.lib.dd_set_streams(self.handle, int(n)), self.lib)

    def stream_count(self) -> int:
        """The handle's current stream count (1 or 2; dd_get_streams)."""
        n = ctypes.c_int()
        _lib.check(self.lib.dd_get_streams(self.handle, ctypes.byref(n)), self.lib)
        return n.value

    def graph_info(self) -> Dict[str, int]:
        """The captured forwards the handle holds (dd_graph_info): ``programs``, their single-stream graph
        ``segments`` in all, and ``multi_stream_execs`` (segments with parallel branches: always 0)."""
        p, s, m = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.dd_graph_info(self.handle, ctypes.byref(p), ctypes.byref(s), ctypes.byref(m)), self.lib)
        k, o = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.dd_graph_nodes(self.handle, ctypes.byref(k), ctypes.byref(o)), self.lib)
        return {"programs": p.value, "segments": s.value, "multi_stream_execs": m.value, "kernel_nodes": k.value,
                "other_nodes": o.value}

    def reset_stats(self):
        _lib.check(self.lib.dd_reset_stats(self.handle), self.lib)

    def kernel_stats(self, kernel: str):
        ms, n, fl = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
        _lib.check(self.lib.dd_kernel_stats(self.handle, kernel.encode(), ctypes.byref(ms), ctypes.byref(n),
                                            ctypes.byref(fl)), self.lib)
        by = ctypes.c_double()
        _lib.check(self.lib.dd_kernel_bytes(self.handle, kernel.encode(), ctypes.byref(by)), self.lib)
        return {"ms": ms.value, "launches": n.value, "flops": fl.value, "bytes": by.value}


class InFlightPlanner:
    """N batches in flight on one device: N handles with the same weights, each a single-stream captured forward
    driven from a stream of its own (dd_set_streams(1): the graph replays on that stream, one hardware queue per
    lane). Consecutive forwards go to consecutive lanes, so one batch's low-occupancy phases (the decoder
    megakernels, the GPT stages, kernel ramps and tails) overlap the next batches' trunks.
    Throughput rises, the latency of each batch grows; the results are those of a single-stream forward, lane for
    lane bit-identical (tests/test_inflight_gpu.py). lanes = 1 is the plain handle (two-stream unless set
    otherwise) on the caller's stream. No reference counterpart (the reference runs one eager forward at a time).

    Outputs are produced on the lane's stream: read them after ``synchronize()`` (or ``wait()``, which makes the
    current stream wait for every lane); each forward first waits for the work already queued on the current
    stream (its inputs)."""

    def __init__(self, config: Optional[TransfuserConfig] = None, state_dict: Optional[Mapping] = None,
                 device: Optional[int] = None, gemm: Optional[str] = None, lanes: int = 2,
                 models: Optional[List[DiffusionDriveModel]] = None, lane_streams: int = 1):
        """``models``: existing handles to use as the lanes (e.g. ``[m] + [m.clone() for _ in ...]``) instead of
        building ``lanes`` handles from ``state_dict``. ``lane_streams`` 2 keeps every lane's two-stream graph
        (three streams per lane with the hand-off: worth it only with $GPU_MAX_HW_QUEUES raised above 4)."""
        if models is not None:
            lanes = len(models)
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self.lanes: List[DiffusionDriveModel] = list(models) if models is not None else \
            [DiffusionDriveModel(config, state_dict, device, gemm) for _ in range(lanes)]
        self.device = self.lanes[0].device
        if lanes > 1:
            for m in self.lanes:
                m.set_streams(lane_streams)
        self.streams = [self._new_stream() for _ in range(lanes)] if lanes > 1 else [None]
        self._next = 0

    # stream primitives (a CPU stand-in planner - bench.py --cpu-plumbing - overrides these three)
    def _new_stream(self):
        return torch.cuda.Stream(torch.device(f"cuda:{self.device}"))

    def _current_stream(self):
        return torch.cuda.current_stream(self.device)

    def _on_stream(self, s):
        return torch.cuda.stream(s)

    def __len__(self):
        return len(self.lanes)

    @property
    def next_index(self) -> int:
        """The lane the next ``next_lane()`` takes."""
        return self._next

    @contextlib.contextmanager
    def next_lane(self):
        """The next lane's model with the current stream set to that lane's stream (which first waits for the
        caller's stream); work issued inside (the forward, a collective on its outputs) is ordered on the lane.
        The round-robin pointer advances only when the body finishes without an exception, so a failed launch
        leaves the lane free for the next batch (the batched runner keeps one pending job per lane)."""
        i = self._next
        s = self.streams[i]
        if s is None:
            yield self.lanes[i]
        else:
            s.wait_stream(self._current_stream())
            with self._on_stream(s):
                yield self.lanes[i]
        self._next = (i + 1) % len(self.lanes)

    def forward(self, features: Dict[str, torch.Tensor], noise: Optional[torch.Tensor] = None,
                steps: Optional[int] = None, heads: bool = False, modes: bool = False) -> Dict[str, torch.Tensor]:
        with self.next_lane() as m:
            return m.forward(features, noise=noise, steps=steps, heads=heads, modes=modes,
                             stream=self._current_stream())

    __call__ = forward

    def wait(self):
        """Make the current stream wait for every lane's queued work."""
        cur = self._current_stream()
        for s in self.streams:
            if s is not None:
                cur.wait_stream(s)

    def synchronize(self):
        for s in self.streams:
            (s or self._current_stream()).synchronize()

    def set_gemm_mode(self, mode: str):
        for m in self.lanes:
            m.set_gemm_mode(mode)

    def numerics_flags(self, clear: bool = True) -> int:
        f = 0
        for m in self.lanes:
            f |= m.numerics_flags(clear)
        return f

    def close(self):
        for m in self.lanes:
            m.close()
