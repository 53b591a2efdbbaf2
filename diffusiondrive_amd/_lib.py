"""ctypes binding of ``libddmi.so`` (the C ABI declared in ``include/ddmi.h``).

The library is the product: there is no fallback. If the shared object is missing or a GPU
is absent, every entry point raises loudly (``DDMIUnavailable``).
"""
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DDMI_LIB", os.path.join(HERE, "libddmi.so"))

c_float_p = ctypes.POINTER(ctypes.c_float)
c_void_p = ctypes.c_void_p


class DDMIUnavailable(RuntimeError):
    """Raised when the native HIP library cannot be loaded."""


class DDMIError(RuntimeError):
    """Raised when a ddmi C-ABI call returns a non-zero status."""


class DDConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int), ("image_arch", ctypes.c_int), ("lidar_arch", ctypes.c_int),
        ("cam_h", ctypes.c_int), ("cam_w", ctypes.c_int), ("lidar_h", ctypes.c_int),
        ("lidar_w", ctypes.c_int), ("lidar_channels", ctypes.c_int), ("num_modes", ctypes.c_int),
        ("num_poses", ctypes.c_int), ("trunc_timestep", ctypes.c_int), ("step_span", ctypes.c_int),
    ]


class DDOutputs(ctypes.Structure):
    _fields_ = [
        ("trajectory", c_void_p), ("poses_reg", c_void_p), ("poses_cls", c_void_p),
        ("bev_semantic_map", c_void_p), ("agent_states", c_void_p), ("agent_labels", c_void_p),
    ]


class DDTrainOutputs(ctypes.Structure):
    _fields_ = [
        ("trajectory", c_void_p), ("poses_reg", c_void_p * 2), ("poses_cls", c_void_p * 2), ("loss", c_void_p),
        ("bev_semantic_map", c_void_p), ("agent_states", c_void_p), ("agent_labels", c_void_p),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "dd_default_config": (None, [ctypes.POINTER(DDConfig)]),
    "dd_create": (ctypes.c_int, [ctypes.POINTER(DDConfig), c_void_p, ctypes.c_size_t, ctypes.c_int,
                                 ctypes.POINTER(c_void_p)]),
    "dd_forward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int, ctypes.c_int,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "dd_forward_ex": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int,
                                     ctypes.c_int, ctypes.POINTER(DDOutputs), c_void_p]),
    "dd_destroy": (ctypes.c_int, [c_void_p]),
    "dd_last_error": (ctypes.c_char_p, []),
    "dd_set_profiling": (ctypes.c_int, [c_void_p, ctypes.c_int]),
    "dd_reset_stats": (ctypes.c_int, [c_void_p]),
    "dd_kernel_stats": (ctypes.c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]),
    "dd_kernel_bytes": (ctypes.c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]),
    "dd_set_seed": (ctypes.c_int, [c_void_p, ctypes.c_ulonglong]),
    "dd_set_seed_at": (ctypes.c_int, [c_void_p, ctypes.c_ulonglong, ctypes.c_ulonglong]),
    "dd_set_graph": (ctypes.c_int, [c_void_p, ctypes.c_int]),
    "dd_set_streams": (ctypes.c_int, [c_void_p, ctypes.c_int]),
    "dd_get_streams": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "dd_graph_info": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int)]),
    "dd_graph_nodes": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "dd_forward_train": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        ctypes.c_int, ctypes.c_float, ctypes.c_float, c_void_p, c_void_p]),
    "dd_bev_semantic_loss": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            c_void_p, c_void_p, c_void_p]),
    "dd_bev_semantic_loss_work": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "dd_set_gemm_mode": (ctypes.c_int, [c_void_p, ctypes.c_int]),
    "dd_set_schedule": (ctypes.c_int, [c_void_p, ctypes.c_int]),
    "dd_get_gemm_mode": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "dd_numerics_flags": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_uint), ctypes.c_int]),
    "dd_tap": (ctypes.c_int, [c_void_p, ctypes.c_char_p, c_void_p, ctypes.c_size_t,
                              ctypes.POINTER(ctypes.c_size_t), c_void_p]),
    "dd_op_last_error": (ctypes.c_char_p, []),
    "dd_op_last_kernel": (ctypes.c_char_p, []),
    "dd_op_mk_linear": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p, ctypes.c_int, c_void_p]),
    "dd_op_bevproj": (ctypes.c_int, [c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_build_camera": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, ctypes.c_int,
                                       ctypes.c_int, c_void_p]),
    "dd_build_lidar": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, c_void_p, ctypes.c_int,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_int, ctypes.c_longlong, c_void_p]),
    "dd_op_conv2d": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_conv2d_x3": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p]),
    "dd_op_stem_pool_x3": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p]),
    "dd_op_stem_pool": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                       c_void_p, ctypes.c_int, c_void_p, c_void_p]),
    "dd_op_stem_pool_nchw": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                            c_void_p, c_void_p, ctypes.c_int, c_void_p, c_void_p]),
    "dd_op_gemm": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                  ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_gemm_batched": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_layernorm": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_softmax_rows": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, c_void_p]),
    "dd_op_bilinear": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                      ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_bilinear_add": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                          ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_maxpool3x3s2": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          c_void_p, c_void_p]),
    "dd_op_avgpool": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, c_void_p, c_void_p]),
    "dd_op_bev_sample_attn": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_mha_small": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p]),
    "dd_op_gpt_attention": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, c_void_p]),
}

EXPORTED = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


def load(path: str = None):
    """Load libddmi.so and bind every C-ABI symbol. Raises DDMIUnavailable if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise DDMIUnavailable(
                f"ddmi native library not found at {p}; build it with `python -m diffusiondrive_amd.build`")
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise DDMIUnavailable(f"cannot load {p}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def check(rc: int, lib=None, op: bool = False):
    if rc != 0:
        lib = lib or load()
        msg = (lib.dd_op_last_error() if op else lib.dd_last_error()) or b""
        raise DDMIError(f"ddmi call failed (rc={rc}): {msg.decode(errors='replace')}")
    return rc
