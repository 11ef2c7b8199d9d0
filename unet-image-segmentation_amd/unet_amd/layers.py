"""Standalone conv_block layer (model/u_net.py:5-26) on the HIP kernels, for eager use of
`conv_block(...)` and per-op tests.  The full model does not use this class: UNetEngine
schedules the same kernels with fused activation views."""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .ops import View
from .params import VarSpec, init_value

BN_EPS = 1e-3
BN_MOMENTUM = 0.99


class ConvBlock:
    def __init__(self, cin: int, cout: int, use_batch_norm: bool = True, name_prefix: str = "conv_block",
                 device=None, seed: int = 2301):
        self.cin, self.cout = int(cin), int(cout)
        self.use_bn = use_batch_norm
        self.name = name_prefix
        dev = torch.device(device or "cuda")
        specs = [VarSpec("depthwise_kernel", (3, 3, cin, 1), True, "glorot_uniform"),
                 VarSpec("pointwise_kernel", (1, 1, cin, cout), True, "glorot_uniform")]
        if use_batch_norm:
            specs += [VarSpec("gamma", (cout,), True, "ones"), VarSpec("beta", (cout,), True, "zeros"),
                      VarSpec("moving_mean", (cout,), False, "zeros"),
                      VarSpec("moving_variance", (cout,), False, "ones")]
        else:
            specs += [VarSpec("bias", (cout,), True, "zeros")]
        self.vars = {s.name: torch.from_numpy(init_value(s, seed, i)).to(dev) for i, s in enumerate(specs)}
        f32 = dict(dtype=torch.float32, device=dev)
        self.scale = torch.empty(cout, **f32)
        self.shift = torch.empty(cout, **f32)
        self.mean = torch.empty(cout, **f32)
        self.rstd = torch.empty(cout, **f32)

    def raw(self, x: torch.Tensor, training: bool):
        """Returns (z, View of relu(bn(z))) for an NHWC input tensor."""
        n, h, w, c = x.shape
        m = n * h * w
        y = torch.empty((n, h, w, c), dtype=torch.float32, device=x.device)
        z = torch.empty((n, h, w, self.cout), dtype=torch.float32, device=x.device)
        ops.dwconv3x3_fwd(View.plain(x.contiguous()), n, h, w, self.vars["depthwise_kernel"], y)
        v = self.vars
        if self.use_bn and training:
            part = torch.zeros(ops.bn_partials_numel(m, self.cout), dtype=torch.float32, device=x.device)
            ops.pointwise_fwd(y, m, c, self.cout, v["pointwise_kernel"], z, part)
            ops.bn_finalize(part, m, self.cout, v["gamma"], v["beta"], BN_EPS, BN_MOMENTUM, v["moving_mean"],
                            v["moving_variance"], True, self.mean, self.rstd, self.scale, self.shift)
        else:
            ops.pointwise_fwd(y, m, c, self.cout, v["pointwise_kernel"], z, None)
            if self.use_bn:
                ops.bn_infer_params(v["gamma"], v["beta"], v["moving_mean"], v["moving_variance"], self.cout,
                                    BN_EPS, self.scale, self.shift)
            else:
                ops.bn_infer_params(None, v["bias"], None, None, self.cout, BN_EPS, self.scale, self.shift)
        return z, View.bnrelu(z, self.scale, self.shift)

    def __call__(self, x: torch.Tensor, training: bool = False) -> torch.Tensor:
        n, h, w, _ = x.shape
        z, view = self.raw(x, training)
        out = torch.empty_like(z)
        return ops.view_materialize(view, n, h, w, out)
