"""keras.optimizers.AdamW as used by the reference (scripts/train.py:59,226), on the HIP
fused multi-tensor kernel.  Keras 3 defaults: learning_rate=0.001, weight_decay=0.004,
beta_1=0.9, beta_2=0.999, epsilon=1e-7; every trainable variable is decayed."""
from __future__ import annotations

import numpy as np
import torch

from . import ops


class AdamW:
    def __init__(self, learning_rate: float = 0.001, weight_decay: float = 0.004, beta_1: float = 0.9,
                 beta_2: float = 0.999, epsilon: float = 1e-7, name: str = "adamw"):
        self.learning_rate = float(learning_rate)
        self.weight_decay = float(weight_decay)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.name = name
        self.iterations = 0
        self._m = None
        self._v = None

    def build(self, params: torch.Tensor):
        if self._m is None or self._m.numel() != params.numel():
            self._m = torch.zeros_like(params)
            self._v = torch.zeros_like(params)

    def alpha(self, step: int) -> float:
        """lr * sqrt(1 - b2^t) / (1 - b1^t), evaluated in float32 as Keras does."""
        t = np.float32(step)
        b1p = np.float32(self.beta_1) ** t
        b2p = np.float32(self.beta_2) ** t
        return float(np.float32(self.learning_rate) * np.sqrt(np.float32(1) - b2p) / (np.float32(1) - b1p))

    def apply(self, params: torch.Tensor, grads: torch.Tensor, grad_scale: float = 1.0):
        """One update of the flat parameter buffer (weight decay, then Adam)."""
        self.build(params)
        step = self.iterations + 1
        ops.adamw_step(params, grads, self._m, self._v, self.learning_rate, self.weight_decay, self.beta_1,
                       self.beta_2, self.epsilon, self.alpha(step), grad_scale)
        self.iterations = step

    def get_config(self):
        return dict(learning_rate=self.learning_rate, weight_decay=self.weight_decay, beta_1=self.beta_1,
                    beta_2=self.beta_2, epsilon=self.epsilon)
