"""Drop-in for the reference's model/u_net.py: the same builder names, signature, defaults,
ValueError and build-time prints, returning a model that runs on the MI355X engine.

Reference: model/u_net.py:5-26 (conv_block), :28-116 (U_NET).
"""
from __future__ import annotations

from typing import Tuple

from unet_amd.params import FILTERS, check_input_size


def conv_block(input_tensor, num_filters: int, kernel_size: int = 3, use_batch_norm: bool = True,
               name_prefix: str = "conv_block"):
    """SeparableConv2D(num_filters, 3, 'same') -> BatchNormalization -> ReLU (model/u_net.py:5-26)
    applied eagerly to an NHWC device tensor with freshly initialised weights and batch
    statistics (what a just-built Keras graph computes in training mode).  Returns
    relu(bn(z)).  Only kernel_size=3 exists on the hot path."""
    if kernel_size != 3:
        raise ValueError("only kernel_size=3 is implemented (the reference only uses 3)")
    from unet_amd.layers import ConvBlock
    blk = ConvBlock(input_tensor.shape[-1], num_filters, use_batch_norm=use_batch_norm, name_prefix=name_prefix,
                    device=input_tensor.device)
    return blk(input_tensor, training=True)


def U_NET(input_size: Tuple[int, int, int], num_classes: int = 1, dropout_rate: float = 0.2,
          use_batch_norm: bool = True, **engine_kwargs):
    """Separable-conv U-Net (model/u_net.py:28-116).  Raises ValueError unless input_size is
    (height, width, channels).  engine_kwargs (filters, device, seed) are engine extras."""
    if len(input_size) != 3:
        raise ValueError("input_size must be a tuple of (height, width, channels)")
    filters = list(engine_kwargs.pop("filters", FILTERS))
    check_input_size(input_size, len(filters))
    print("Building Encoder...")
    for i, f in enumerate(filters):
        print(f"  Encoder Stage {i + 1}, Filters: {f}")
    print("Building Bottleneck...")
    print(f"  Bottleneck Filters: {filters[-1] * 2}")
    print("Building Decoder...")
    for i, f in enumerate(reversed(filters)):
        print(f"  Decoder Stage {len(filters) - i}, Filters: {f}")
    print("Building Output Layer...")
    from unet_amd.model import UNetModel
    model = UNetModel(input_size, num_classes, dropout_rate, use_batch_norm, filters=filters, **engine_kwargs)
    print("U-Net model built successfully.")
    return model


def unet(input_size: Tuple[int, int, int], num_classes: int = 1, **kwargs):
    """`unet(input_size, num_classes)` builder named by the north star; alias of U_NET."""
    return U_NET(input_size, num_classes, **kwargs)
