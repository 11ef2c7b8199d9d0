"""Drop-in for the reference's utils/metrics.py (dice_coef :6-39, iou_coef :41-62), computed
by the HIP dice kernel on device tensors.  SMOOTH = K.epsilon() = 1e-7."""
from unet_amd.metrics import SMOOTH, dice_coef, iou_coef  # noqa: F401

__all__ = ["SMOOTH", "dice_coef", "iou_coef"]
