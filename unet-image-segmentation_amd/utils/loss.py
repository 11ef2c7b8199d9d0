"""Drop-in for the reference's utils/loss.py (dice_loss :9-29, iou_loss :31-45, jaccard_loss
:48).  iou_loss computes the intended 1 - iou_coef (the reference forgets to import iou_coef,
so its iou_loss raises NameError when called)."""
from unet_amd.metrics import SMOOTH, dice_loss, iou_loss, jaccard_loss  # noqa: F401

__all__ = ["SMOOTH", "dice_loss", "iou_loss", "jaccard_loss"]
