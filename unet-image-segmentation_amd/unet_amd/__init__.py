"""unet_amd: MI355X-native engine for the separable-conv U-Net hot path of
planck-epoch/unet-image-segmentation (HIP kernels for gfx950 behind a C-ABI,
include/unet_hip.h; PyTorch-ROCm only for device memory, streams and RCCL)."""
import os as _os

# Kernel arguments in device memory: the step is ~210 dependent launches, and reading each launch's
# arguments from host memory lengthened every kernel boundary (step A/B on MI355X: 1390 vs 1368
# img/s, profiles/r2x_ab.log).  Read by the HIP runtime when it initialises, so it is set here,
# before any device call; an explicit setting in the environment wins.  Import this package before
# anything initialises HIP (torch.cuda.init(), a device tensor): afterwards the setting is ignored.
if "HIP_FORCE_DEV_KERNARG" not in _os.environ:
    _os.environ["HIP_FORCE_DEV_KERNARG"] = "1"
    _torch = __import__("sys").modules.get("torch")
    if _torch is not None and _torch.cuda.is_initialized():
        import warnings as _warnings
        _warnings.warn("unet_amd imported after HIP was initialised: HIP_FORCE_DEV_KERNARG=1 has no "
                       "effect in this process (kernel arguments stay in host memory, ~1.5 % slower "
                       "steps); import unet_amd first or export the variable", RuntimeWarning)
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
