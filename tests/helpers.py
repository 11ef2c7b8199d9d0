"""Shared test helpers (host <-> device, error metrics, oracle-side view restatements)."""
from __future__ import annotations

import numpy as np

from oracle import keras_ops as K


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32))).cuda()


def host(t):
    return t.detach().cpu().numpy().astype(np.float64)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def norm_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def f32(a):
    """Round an array to float32 and return it as float64 (what the device sees)."""
    return np.asarray(a, np.float32).astype(np.float64)


def bn_affine(rng, c, allow_negative=True):
    gamma = 1.0 + 0.3 * rng.standard_normal(c)
    if allow_negative:
        gamma[::5] *= -1.0
    beta = 0.2 * rng.standard_normal(c)
    return f32(gamma), f32(beta)


def view_value(mode, src0, sc0=None, sh0=None, src1=None, sc1=None, sh1=None, drop_rate=0.0, drop_seed=0):
    """Oracle restatement of a unet_view's logical tensor (include/unet_hip.h)."""
    if mode == 0:
        x = src0
    elif mode == 1:
        x = K.relu(src0 * sc0 + sh0)
    elif mode == 2:
        x = K.maxpool2(K.relu(src0 * sc0 + sh0))
    else:
        x = np.concatenate([src0, K.relu(src1 * sc1 + sh1)], axis=-1)
    if drop_rate > 0:
        x = x * K.dropout_mult(drop_seed, x.shape, drop_rate, np.float64)
    return x
