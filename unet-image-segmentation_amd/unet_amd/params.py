"""Variable inventory of the reference U-Net (model/u_net.py:28-116) in Keras `model.weights`
order, with Keras layouts, names and initializers, and the flat HBM layout the engine uses.

All trainable variables live in ONE flat float32 buffer (each tensor 256-byte aligned), so
gradients are one buffer too: the data-parallel all-reduce and the fused AdamW each touch a
single allocation.  BatchNorm moving statistics live in a second flat buffer.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np

FILTERS = (64, 128, 256, 512)  # model/u_net.py:57
ALIGN = 64  # floats (256 B)


@dataclass(frozen=True)
class VarSpec:
    name: str
    shape: Tuple[int, ...]
    trainable: bool
    init: str  # glorot_uniform | zeros | ones

    @property
    def size(self) -> int:
        return int(np.prod(self.shape))


def check_input_size(input_size: Sequence[int], depth: int = 4) -> Tuple[int, int, int]:
    """model/u_net.py:52-53 raises ValueError unless input_size is (H, W, C).  H and W must be
    divisible by 2**depth or the decoder concat shapes mismatch."""
    if input_size is None or len(tuple(input_size)) != 3:
        raise ValueError("input_size must be a tuple of (height, width, channels)")
    h, w, c = (int(v) for v in input_size)
    if h <= 0 or w <= 0 or c <= 0:
        raise ValueError(f"input_size must be positive, got {tuple(input_size)}")
    div = 2 ** depth
    if h % div or w % div:
        raise ValueError(f"height and width must be divisible by {div} (got {h}x{w}): the skip concatenations "
                         f"of the decoder need matching shapes")
    return h, w, c


def unet_variables(input_channels: int = 3, num_classes: int = 1, use_batch_norm: bool = True,
                   filters: Sequence[int] = FILTERS) -> List[VarSpec]:
    """Every variable of U_NET in Keras creation order (layer order of the functional graph)."""
    out: List[VarSpec] = []

    def conv_block(prefix: str, cin: int, cout: int):
        out.append(VarSpec(f"{prefix}_sepconv/depthwise_kernel", (3, 3, cin, 1), True, "glorot_uniform"))
        out.append(VarSpec(f"{prefix}_sepconv/pointwise_kernel", (1, 1, cin, cout), True, "glorot_uniform"))
        if not use_batch_norm:
            out.append(VarSpec(f"{prefix}_sepconv/bias", (cout,), True, "zeros"))
        else:
            out.append(VarSpec(f"{prefix}_bn/gamma", (cout,), True, "ones"))
            out.append(VarSpec(f"{prefix}_bn/beta", (cout,), True, "zeros"))
            out.append(VarSpec(f"{prefix}_bn/moving_mean", (cout,), False, "zeros"))
            out.append(VarSpec(f"{prefix}_bn/moving_variance", (cout,), False, "ones"))

    c = input_channels
    for i, f in enumerate(filters):
        conv_block(f"enc{i + 1}_block1", c, f)
        conv_block(f"enc{i + 1}_block2", f, f)
        c = f
    bn = filters[-1] * 2  # model/u_net.py:73
    conv_block("bneck_block1", c, bn)
    conv_block("bneck_block2", bn, bn)
    c = bn
    for i, f in enumerate(reversed(filters)):
        stage = len(filters) - i
        out.append(VarSpec(f"dec{stage}_upsample/kernel", (2, 2, f, c), True, "glorot_uniform"))
        out.append(VarSpec(f"dec{stage}_upsample/bias", (f,), True, "zeros"))
        conv_block(f"dec{stage}_block1", 2 * f, f)
        conv_block(f"dec{stage}_block2", f, f)
        c = f
    out.append(VarSpec("output_mask/kernel", (1, 1, c, num_classes), True, "glorot_uniform"))
    out.append(VarSpec("output_mask/bias", (num_classes,), True, "zeros"))
    return out


def compute_fans(shape: Tuple[int, ...]) -> Tuple[int, int]:
    """keras.initializers compute_fans: receptive field = prod(shape[:-2])."""
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[:-2]))
    return shape[-2] * rf, shape[-1] * rf


_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def portable_uniform(seed: int, n: int) -> np.ndarray:
    """n doubles in [0, 1) from splitmix64(seed + i*golden) >> 11 (documented, portable stream)."""
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GOLDEN)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def init_value(spec: VarSpec, seed: int, index: int) -> np.ndarray:
    """Keras default initial value of a variable (glorot_uniform limit sqrt(6/(fan_in+fan_out)),
    zeros, ones).  Random draws come from the portable stream, not TF's RNG."""
    if spec.init == "zeros":
        return np.zeros(spec.shape, np.float32)
    if spec.init == "ones":
        return np.ones(spec.shape, np.float32)
    fan_in, fan_out = compute_fans(spec.shape)
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    u = portable_uniform(seed * 1000003 + index, spec.size)
    return ((2.0 * u - 1.0) * limit).astype(np.float32).reshape(spec.shape)


def init_weights(specs: List[VarSpec], seed: int = 2301) -> Dict[str, np.ndarray]:
    return {s.name: init_value(s, seed, i) for i, s in enumerate(specs)}


@dataclass
class FlatLayout:
    offsets: Dict[str, int]
    total: int


def flat_layout(specs: List[VarSpec], trainable: bool) -> FlatLayout:
    offs, cur = {}, 0
    for s in specs:
        if s.trainable != trainable:
            continue
        offs[s.name] = cur
        cur += (s.size + ALIGN - 1) // ALIGN * ALIGN
    return FlatLayout(offs, max(cur, ALIGN))


def count_params(specs: List[VarSpec]) -> Tuple[int, int]:
    tr = sum(s.size for s in specs if s.trainable)
    nt = sum(s.size for s in specs if not s.trainable)
    return tr, nt
