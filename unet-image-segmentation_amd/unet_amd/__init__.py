"""unet_amd: MI355X-native engine for the separable-conv U-Net hot path of
planck-epoch/unet-image-segmentation (HIP kernels for gfx950 behind a C-ABI,
include/unet_hip.h; PyTorch-ROCm only for device memory, streams and RCCL)."""
from ._lib import UnetHipError, load as load_library  # noqa: F401
from .params import FILTERS, unet_variables  # noqa: F401

__all__ = ["UnetHipError", "load_library", "FILTERS", "unet_variables"]


def __getattr__(name):
    # device-dependent pieces are imported lazily so host-only tools can import the package
    if name in ("UNetEngine",):
        from .engine import UNetEngine
        return UNetEngine
    if name in ("UNetModel",):
        from .model import UNetModel
        return UNetModel
    if name in ("AdamW",):
        from .optim import AdamW
        return AdamW
    if name in ("MeanIoU",):
        from .metrics import MeanIoU
        return MeanIoU
    raise AttributeError(name)
