"""Losses and metrics of the reference on HIP kernels.

  dice_coef / iou_coef           utils/metrics.py:6-62
  dice_loss / iou_loss / jaccard utils/loss.py:9-48 (iou_loss is broken in the reference: it
                                 calls iou_coef without importing it, utils/loss.py:4,43; here it
                                 computes the intended 1 - iou_coef)
  MeanIoU                        keras.metrics.MeanIoU (scripts/train.py:231, benchmark.py:237)
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import ops

SMOOTH = 1e-7  # K.epsilon()


def as_device_tensor(t, device=None) -> torch.Tensor:
    if isinstance(t, torch.Tensor):
        if not t.is_cuda:
            t = t.to(device or "cuda")
        return t.to(torch.float32).contiguous()
    return torch.as_tensor(np.asarray(t, dtype=np.float32), device=device or "cuda").contiguous()


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    if t.dim() == 3:  # (B, H, W) -> (B, H, W, 1)
        t = t.unsqueeze(-1)
    if t.dim() != 4:
        raise ValueError(f"expected (batch, H, W, C) tensors, got shape {tuple(t.shape)}")
    return t


def dice_sums(y_true, y_pred, smooth: float = SMOOTH) -> torch.Tensor:
    """Device vector [1 - mean dice, mean dice, mean iou] of (y_true, y_pred) (B, H, W, C)."""
    yp = _nhwc(as_device_tensor(y_pred))
    yt = _nhwc(as_device_tensor(y_true, yp.device))
    if yt.shape != yp.shape:
        raise ValueError(f"y_true {tuple(yt.shape)} and y_pred {tuple(yp.shape)} differ")
    b, h, w, c = yp.shape
    res = torch.empty(3, dtype=torch.float32, device=yp.device)
    ops.dice_fwd(yt, yp, b, h * w, c, smooth, None, res)
    return res


def dice_coef(y_true, y_pred, smooth: float = SMOOTH) -> torch.Tensor:
    return dice_sums(y_true, y_pred, smooth)[1]


def iou_coef(y_true, y_pred, smooth: float = SMOOTH) -> torch.Tensor:
    return dice_sums(y_true, y_pred, smooth)[2]


def dice_loss(y_true, y_pred) -> torch.Tensor:
    return dice_sums(y_true, y_pred)[0]


def iou_loss(y_true, y_pred, smooth: float = SMOOTH) -> torch.Tensor:
    return 1.0 - dice_sums(y_true, y_pred, smooth)[2]


jaccard_loss = iou_loss


class MeanIoU:
    """keras.metrics.MeanIoU(num_classes): confusion matrix over flattened labels.

    threshold=None reproduces Keras' cast semantics on raw probabilities (float -> int64
    truncation; how the reference's training metric sees sigmoid outputs); pass a
    threshold to score binarised predictions as scripts/benchmark.py:260 does."""

    def __init__(self, num_classes: int, name: str = "mean_io_u", threshold: Optional[float] = None,
                 device=None):
        self.num_classes = int(num_classes)
        self.name = name
        self.threshold = threshold
        self.device = torch.device(device or "cuda")
        self.confusion = torch.zeros(self.num_classes * self.num_classes, dtype=torch.int64, device=self.device)

    def update_state(self, y_true, y_pred, threshold: Optional[float] = None):
        yp = as_device_tensor(y_pred, self.device)
        yt = as_device_tensor(y_true, self.device)
        thr = self.threshold if threshold is None else threshold
        ops.meaniou_update(yt.reshape(-1), yp.reshape(-1), self.num_classes, thr, self.confusion)

    def confusion_matrix(self) -> np.ndarray:
        return self.confusion.cpu().numpy().reshape(self.num_classes, self.num_classes)

    def result(self) -> float:
        cm = self.confusion_matrix().astype(np.float64)
        tp = np.diag(cm)
        den = cm.sum(axis=0) + cm.sum(axis=1) - tp
        valid = den != 0
        if not valid.any():
            return 0.0
        return float((tp[valid] / den[valid]).sum() / valid.sum())

    def reset_state(self):
        self.confusion.zero_()

    def all_reduce(self, group=None):
        """Sum confusion counts over data-parallel ranks."""
        import torch.distributed as dist
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.confusion, group=group)
