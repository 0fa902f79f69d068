"""ctypes binding of libyolo_hip.so (C ABI declared in include/yolo_hip.h).

The shared library is built in-tree by `make` (or __graft_entry__.build()) next
to this file. Loading it does not touch the GPU; every compute entry point
needs a HIP device. torch is imported before the library is opened so both use
PyTorch's HIP runtime. There is deliberately no fallback: if the library cannot
be loaded, GPU inference raises.
"""
import ctypes
import os
from ctypes import POINTER, byref, c_char_p, c_double, c_float, c_int, c_size_t, c_void_p

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libyolo_hip.so")
# experiments only: YH_LIB=<path> loads another build of the same library
if os.environ.get("YH_LIB"):
    LIB_PATH = os.environ["YH_LIB"]

YH_F32, YH_F16, YH_BF16 = 0, 1, 2
ABI_VERSION = 5


class YhVariant(ctypes.Structure):
    _fields_ = [
        ("width", c_int * 6),
        ("depth", c_int * 6),
        ("csp", c_int * 2),
        ("num_classes", c_int),
    ]


# name -> (restype, argtypes); mirrors include/yolo_hip.h
_PROTOS = {
    "yh_abi_version": (c_int, []),
    "yh_last_error": (c_char_p, []),
    "yh_create": (c_int, [POINTER(YhVariant), c_int, c_int, POINTER(c_void_p)]),
    "yh_destroy": (None, [c_void_p]),
    "yh_conv_count": (c_int, [c_void_p]),
    "yh_conv_info": (c_int, [c_void_p, c_int, POINTER(c_char_p), POINTER(c_int), POINTER(c_int),
                             POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "yh_load_conv": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_double]),
    "yh_num_anchors": (c_int, [c_void_p, c_int, c_int, POINTER(c_int)]),
    "yh_workspace_bytes": (c_int, [c_void_p, c_int, c_int, c_int, POINTER(c_size_t)]),
    "yh_reserve": (c_int, [c_void_p, c_int, c_int, c_int]),
    "yh_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "yh_forward_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "yh_nms_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "yh_nms": (c_int, [c_int, c_void_p, c_int, c_int, c_int, c_float, c_double, c_int, c_int, c_float,
                       c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "yh_profile_enable": (c_int, [c_void_p, c_int]),
    "yh_profile_reset": (c_int, [c_void_p]),
    "yh_op_count": (c_int, [c_void_p]),
    "yh_op_info": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_char_p), POINTER(c_int),
                           POINTER(c_double), POINTER(c_double), POINTER(c_double), POINTER(c_int)]),
    "yh_set_graph": (c_int, [c_void_p, c_int]),
    "yh_op_kernel": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_char_p)]),
    "yh_force_conv_kernel": (c_int, [c_void_p, c_int]),
    "yh_unit_count": (c_int, [c_void_p, c_int, c_int, c_int]),
    "yh_unit_info": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_int), POINTER(c_int), POINTER(c_int),
                             POINTER(c_double), POINTER(c_int)]),
    "yh_nms_host": (c_int, [c_int, c_void_p, c_int, c_int, c_int, c_float, c_double, c_int, c_int, c_float,
                            c_void_p, c_void_p, c_int]),
    "yh_letterbox_geometry": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "yh_letterbox": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "yh_letterbox_host": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int]),
    "yh_resize_linear_host": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "yh_debug_op_desc": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_char_p, c_size_t]),
    "yh_debug_run_ops": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "yh_debug_operand": (c_int, [c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p]),
}

_lib = None


def lib():
    """Load (once) and return the ctypes library; raises if it is missing."""
    global _lib
    if _lib is None:
        # PyTorch-ROCm ships its own libamdhip64.so.7. Importing torch first makes the
        # dynamic loader resolve our DT_NEEDED libamdhip64.so.7 to that same runtime,
        # so the library and torch share one HIP runtime (streams, graphs, memory).
        # Loading ours first would bring in /opt/rocm's copy next to torch's.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"yolo_hip: {LIB_PATH} not found; build it with `make` (or __graft_entry__.build())")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        ver = handle.yh_abi_version()
        if ver != ABI_VERSION:
            raise RuntimeError(f"yolo_hip: ABI version {ver}, expected {ABI_VERSION}")
        _lib = handle
    return _lib


def check(rc, what=""):
    """Raise RuntimeError carrying yh_last_error() for a negative status code."""
    if rc != 0:
        msg = lib().yh_last_error()
        msg = msg.decode() if msg else ""
        raise RuntimeError(f"yolo_hip{': ' + what if what else ''}: {msg} (status {rc})")


__all__ = ["lib", "check", "YhVariant", "YH_F32", "YH_F16", "YH_BF16", "LIB_PATH",
           "byref", "c_void_p", "c_int", "c_char_p", "c_double", "c_size_t"]
