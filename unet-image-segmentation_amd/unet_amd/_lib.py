"""ctypes binding of libunet_hip.so (the C-ABI declared in include/unet_hip.h).

This is the only way the host code reaches the HIP kernels.  There is no CPU fallback:
if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_int32, c_int64, c_size_t, c_uint64, c_void_p, c_char_p
from pathlib import Path

LIB_NAME = "libunet_hip.so"
LIB_PATH = Path(os.environ.get("UNET_HIP_LIB", Path(__file__).with_name(LIB_NAME)))
ABI_VERSION = 12
SPLIT_MAX_SEGS = 64  # UNET_SPLIT_MAX_SEGS

VIEW_PLAIN, VIEW_BNRELU, VIEW_POOL_BNRELU, VIEW_CONCAT = 0, 1, 2, 3
LOSS_DICE, LOSS_IOU = 0, 1


class UnetView(ctypes.Structure):
    """Mirror of `unet_view` (include/unet_hip.h)."""

    _fields_ = [
        ("mode", c_int32),
        ("c0", c_int32),
        ("c1", c_int32),
        ("reserved0", c_int32),
        ("src0", c_void_p),
        ("scale0", c_void_p),
        ("shift0", c_void_p),
        ("src1", c_void_p),
        ("scale1", c_void_p),
        ("shift1", c_void_p),
        ("drop_rate", c_float),
        ("reserved1", c_int32),
        ("drop_seed", c_uint64),
    ]


_VP = POINTER(UnetView)
P = c_void_p
# name -> (restype, argtypes); exactly the entry points of include/unet_hip.h
SIGNATURES = {
    "unet_abi_version": (c_int, []),
    "unet_copy_strided": (c_int, [P, c_int64, c_int, c_int64, P, c_int64, P]),
    "unet_last_error": (c_char_p, []),
    "unet_event_create": (c_int, [POINTER(c_void_p)]),
    "unet_event_destroy": (c_int, [P]),
    "unet_stream_wait_stream": (c_int, [P, P, P]),
    "unet_view_materialize": (c_int, [_VP, c_int, c_int, c_int, P, P]),
    "unet_dwconv3x3_fwd": (c_int, [_VP, c_int, c_int, c_int, P, P, P]),
    "unet_dwconv3x3_bwd_data": (c_int, [_VP, c_int, c_int, c_int, P, P, P, P, P]),
    "unet_dwconv3x3_bwd_data_bnstats_slabs": (c_int, [_VP, c_int, c_int, c_int]),
    "unet_dwconv3x3_bwd_data_bnstats": (c_int, [_VP, c_int, c_int, c_int, P, P, P, P, P, P, P]),
    "unet_dwconv3x3_bwd_data_bnstats_dwf": (c_int, [_VP, c_int, c_int, c_int, P, P, P, P, P, P, P, P]),
    "unet_reduce_slabs": (c_int, [P, c_int, c_int64, P, P]),
    "unet_dwconv3x3_bwd_filter_workspace": (c_size_t, [c_int, c_int, c_int, c_int]),
    "unet_dwconv3x3_bwd_filter": (c_int, [_VP, c_int, c_int, c_int, P, P, P, c_size_t, P]),
    "unet_bn_partials_size": (c_size_t, [c_int64, c_int]),
    "unet_pointwise_fwd": (c_int, [P, c_int64, c_int, c_int, P, P, P, P]),
    "unet_pointwise_fwd_x3": (c_int, [P, c_int64, c_int, c_int, P, P, P, P, P]),
    "unet_pointwise_bwd_data": (c_int, [P, c_int64, c_int, c_int, P, P, P]),
    "unet_pointwise_bwd_filter_workspace": (c_size_t, [c_int64, c_int, c_int]),
    "unet_pointwise_bwd_filter": (c_int, [P, P, c_int64, c_int, c_int, P, P, c_size_t, P]),
    "unet_sepconv_fwd_supported": (c_int, [_VP, c_int, c_int, c_int, c_int]),
    "unet_sepconv_fwd": (c_int, [_VP, c_int, c_int, c_int, P, c_int, P, P, P, P, P, P, P, P]),
    "unet_split_x3": (c_int, [P, P, c_int, P, P]),
    "unet_split_x3_keep": (c_int, [P, P, c_int, P, P]),
    "unet_split_x3_mixed": (c_int, [P, P, c_int, P, P]),
    "unet_pool_select": (c_int, [P, c_int, c_int, c_int, c_int, P, P, P]),
    "unet_sepconv_bwd_filter_supported": (c_int, [_VP, c_int, c_int, c_int, c_int]),
    "unet_sepconv_bwd_filter_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "unet_sepconv_bwd_filter": (c_int, [_VP, c_int, c_int, c_int, P, P, P, c_int, P, P, P, c_size_t, P]),
    "unet_sepconv_bwd_fused": (c_int, [_VP, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, c_int, P, P, P, P,
                                       c_size_t, P]),
    "unet_sepconv_set_schedule": (c_int, [c_int]),
    "unet_bn_finalize": (c_int, [P, c_int64, c_int, P, P, c_float, c_float, P, P, c_int, P, P, P, P, P]),
    "unet_bn_moments": (c_int, [P, c_int64, c_int, P, P]),
    "unet_bn_finalize_moments": (c_int, [P, c_int, c_int, P, P, c_float, c_float, P, P, c_int, P, P, P, P, P]),
    "unet_bn_bwd_coef": (c_int, [P, c_int64, c_int, c_int, P, P, P, P]),
    "unet_bn_infer_params": (c_int, [P, P, P, P, c_int, c_float, P, P, P]),
    "unet_bn_relu_bwd_workspace": (c_size_t, [c_int64, c_int]),
    "unet_bn_relu_bwd": (c_int, [P, P, c_int64, c_int, P, P, P, P, c_int, c_float, c_uint64, P, P, P, P,
                                 c_size_t, P]),
    "unet_bn_stats_partials_size": (c_size_t, [c_int, c_int]),
    "unet_bn_relu_bwd_stats_finish": (c_int, [P, c_int, c_int64, c_int, P, P, c_int, P, P, P, P]),
    "unet_bn_relu_bwd_stats": (c_int, [P, P, c_int64, c_int, P, P, P, P, c_int, c_float, c_uint64, P, P, P, P,
                                       c_size_t, P]),
    "unet_pointwise_bwd_data_bnrelu": (c_int, [P, P, c_int64, c_int, c_int, P, P, P, P, c_float, c_uint64, P, P,
                                               P]),
    "unet_pointwise_bwd_data_bnrelu_x3": (c_int, [P, P, c_int64, c_int, c_int, P, P, P, P, P, c_float, c_uint64, P,
                                                  P, P]),
    "unet_pointwise_bwd_data_bnrelu_wgrad_workspace": (c_size_t, [c_int64, c_int, c_int]),
    "unet_pointwise_bwd_data_bnrelu_wgrad": (c_int, [P, P, c_int64, c_int, c_int, P, P, P, P, P, P, P, P, c_size_t,
                                                     P]),
    "unet_image_block_bwd_wgrad_workspace": (c_size_t, [c_int, c_int, c_int, c_int]),
    "unet_image_block_bwd_wgrad": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P,
                                           c_size_t, P]),
    "unet_conv_transpose2x2_fwd": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P]),
    "unet_conv_transpose2x2_fwd_x3": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "unet_conv_transpose2x2_bwd_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "unet_conv_transpose2x2_bwd": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P, P, P, c_size_t, P]),
    "unet_conv_transpose2x2_bwd_data_bnstats_slabs": (c_int, [_VP, c_int, c_int, c_int, c_int]),
    "unet_conv_transpose2x2_bwd_data_bnstats": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P, P, P, P]),
    "unet_conv_transpose2x2_bwd_data_bnstats_x3": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P, P, P, P,
                                                          P]),
    "unet_head_fwd": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P]),
    "unet_dice_workspace": (c_size_t, [c_int, c_int64, c_int]),
    "unet_dice_fwd": (c_int, [P, P, c_int, c_int64, c_int, c_float, P, P, P, c_size_t, P]),
    "unet_head_bwd_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "unet_head_bwd_bnstats_slabs": (c_int, [_VP, c_int, c_int, c_int, c_int]),
    "unet_head_bwd_bnstats": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P, c_float, c_int, c_float, P, P, P, P, P,
                                      P, P, P, c_size_t, P]),
    "unet_head_bwd": (c_int, [_VP, c_int, c_int, c_int, c_int, P, P, P, P, c_float, c_int, c_float, P, P, P, P, c_size_t,
                              P]),
    "unet_meaniou_update": (c_int, [P, P, c_int64, c_int, c_float, P, P]),
    "unet_adamw_step": (c_int, [P, P, P, P, c_int64, c_float, c_float, c_float, c_float, c_float, c_float, c_float,
                                P]),
}

_lib = None


class UnetHipError(RuntimeError):
    pass


def load(path: os.PathLike | str | None = None):
    """Load (once) and return the ctypes library.  Raises if it is missing: the product path
    has no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise UnetHipError(
            f"{p} not found: build it with `python __graft_entry__.py` (build()) or "
            f"`make -C unet-image-segmentation_amd/csrc`; there is no CPU fallback")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.unet_abi_version()
    if v != ABI_VERSION:
        raise UnetHipError(f"{p}: ABI version {v} != expected {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def call(name: str, *args) -> None:
    """Call an int-returning entry point; raise UnetHipError with unet_last_error() on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.unet_last_error().decode(errors="replace")
        kind = "invalid argument" if rc < 0 else f"hipError {rc}"
        raise UnetHipError(f"{name} failed ({kind}): {msg}")


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
