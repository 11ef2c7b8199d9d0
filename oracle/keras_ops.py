"""CPU oracle: NumPy restatement of the reference hot path's op semantics.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the CPU baseline.  The product path (``unet_amd``) never calls it.

PARITY UNPINNED: the reference (planck-epoch/unet-image-segmentation) ships no
tests, golden vectors or fixtures, and its arithmetic lives in an un-vendored,
unpinned TensorFlow/Keras that is not importable here (plain
ModuleNotFoundError, not a permission denial).  This module
restates the Keras 3 semantics of each op the reference's files call, and is
cross-checked against an independent torch-CPU float64 restatement in
``tests/test_oracle.py``; its outputs are frozen as fixtures in
``tests/golden/`` (made by ``tests/golden/make_golden.py``).

Every function works in the dtype of its inputs (float64 for parity checks,
float32 for the CPU baseline).  Layouts are the reference's: NHWC activations,
Keras weight layouts.
"""
from __future__ import annotations

import numpy as np

# Keras backend.epsilon(); the reference's SMOOTH (utils/metrics.py:4, utils/loss.py:7)
SMOOTH = 1e-7
# keras.layers.BatchNormalization defaults (model/u_net.py:23 uses BatchNormalization())
BN_EPS = 1e-3
BN_MOMENTUM = 0.99


# ----------------------------------------------------------------------------- dropout ---
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def dropout_mult(seed: int, shape, rate: float, dtype=np.float64) -> np.ndarray:
    """Multiplier of keras.layers.Dropout(rate) in training (model/u_net.py:77-78, 97-98):
    keep with probability 1-rate, scale kept values by 1/(1-rate).  The Bernoulli draw is
    the engine's documented counter-based generator (TF's RNG stream is not reproducible
    across frameworks): for the linear NHWC index i of an element,
    h = splitmix64(seed + (i >> 2)*golden), u(i) = ((h >> 16 (i & 3)) & 0xffff) / 2^16,
    keep iff u >= rate (csrc/common.h: drop_mult)."""
    if rate <= 0.0:
        return np.ones(shape, dtype=dtype)
    n = int(np.prod(shape))
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = splitmix64(np.uint64(seed) + (idx >> np.uint64(2)) * _GOLDEN)
    bits = (h >> (np.uint64(16) * (idx & np.uint64(3)))) & np.uint64(0xFFFF)
    u32 = bits.astype(np.float32) * np.float32(1.0 / 65536.0)
    keep = u32 >= np.float32(rate)
    inv_keep = np.float32(1.0) / (np.float32(1.0) - np.float32(rate))
    return np.where(keep, inv_keep, 0).astype(dtype).reshape(shape)


# ------------------------------------------------------------------ SeparableConv2D ------
def depthwise3x3(x: np.ndarray, dk: np.ndarray) -> np.ndarray:
    """DepthwiseConv2dNative of SeparableConv2D(f, 3, padding='same') (model/u_net.py:14-20):
    y[n,h,w,c] = sum_{i,j} x[n,h+i-1,w+j-1,c] * dk[i,j,c,0], zero padding (cross-correlation)."""
    N, H, W, C = x.shape
    xp = np.zeros((N, H + 2, W + 2, C), dtype=x.dtype)
    xp[:, 1:-1, 1:-1, :] = x
    y = np.zeros_like(x)
    for i in range(3):
        for j in range(3):
            y += xp[:, i:i + H, j:j + W, :] * dk[i, j, :, 0]
    return y


def depthwise3x3_bwd(x: np.ndarray, dk: np.ndarray, dy: np.ndarray):
    """Gradients of depthwise3x3 w.r.t. its input and its (3,3,C,1) kernel."""
    N, H, W, C = x.shape
    xp = np.zeros((N, H + 2, W + 2, C), dtype=x.dtype)
    xp[:, 1:-1, 1:-1, :] = x
    dxp = np.zeros_like(xp)
    ddk = np.zeros_like(dk)
    for i in range(3):
        for j in range(3):
            dxp[:, i:i + H, j:j + W, :] += dy * dk[i, j, :, 0]
            ddk[i, j, :, 0] = np.einsum("nhwc,nhwc->c", xp[:, i:i + H, j:j + W, :], dy)
    return dxp[:, 1:-1, 1:-1, :], ddk


def pointwise(y: np.ndarray, pk: np.ndarray) -> np.ndarray:
    """Pointwise stage of SeparableConv2D: z = y . pk[0,0] (Keras pointwise_kernel (1,1,Cin,Cout))."""
    N, H, W, C = y.shape
    return (y.reshape(-1, C) @ pk[0, 0]).reshape(N, H, W, -1)


def pointwise_bwd(y: np.ndarray, pk: np.ndarray, dz: np.ndarray):
    N, H, W, C = y.shape
    dz2 = dz.reshape(-1, dz.shape[-1])
    dy = (dz2 @ pk[0, 0].T).reshape(y.shape)
    dpk = (y.reshape(-1, C).T @ dz2)[None, None]
    return dy, dpk


# ----------------------------------------------------------------- BatchNormalization ----
def bn_train(z: np.ndarray, gamma, beta, eps=BN_EPS):
    """Keras 3 BatchNormalization(training=True) (model/u_net.py:22-23): tf.nn.moments over
    (N,H,W) -> mean, biased variance; out = z*inv + (beta - mean*inv), inv = gamma*rsqrt(var+eps)."""
    C = z.shape[-1]
    z2 = z.reshape(-1, C)
    mean = z2.mean(axis=0)
    var = ((z2 - mean) ** 2).mean(axis=0)
    inv = gamma / np.sqrt(var + eps)
    out = z * inv + (beta - mean * inv)
    return out, mean, var


def bn_moving_update(mm, mv, mean, var, momentum=BN_MOMENTUM):
    """moving = moving*momentum + batch*(1-momentum), batch variance biased (Keras 3)."""
    return mm * momentum + mean * (1 - momentum), mv * momentum + var * (1 - momentum)


def bn_infer(z, gamma, beta, mm, mv, eps=BN_EPS):
    inv = gamma / np.sqrt(mv + eps)
    return z * inv + (beta - mm * inv)


def bn_relu_bwd(da, z, gamma, beta, mean, var, eps=BN_EPS, drop=None):
    """Backward of a = [dropout](relu(bn_train(z))).  Returns dz, dgamma, dbeta."""
    C = z.shape[-1]
    rstd = 1.0 / np.sqrt(var + eps)
    inv = gamma * rstd
    pre = z * inv + (beta - mean * inv)
    g = da if drop is None else da * drop
    g = np.where(pre > 0, g, 0).reshape(-1, C)
    xhat = ((z - mean) * rstd).reshape(-1, C)
    M = g.shape[0]
    dbeta = g.sum(axis=0)
    dgamma = (g * xhat).sum(axis=0)
    dz = inv * (g - dbeta / M - xhat * dgamma / M)
    return dz.reshape(z.shape), dgamma, dbeta


def relu(x):
    return np.maximum(x, 0)


# ----------------------------------------------------------------------- MaxPool / concat -
def maxpool2(a: np.ndarray) -> np.ndarray:
    """MaxPooling2D((2,2)) 'valid', stride 2 (model/u_net.py:69)."""
    N, H, W, C = a.shape
    return a[:, :H // 2 * 2, :W // 2 * 2].reshape(N, H // 2, 2, W // 2, 2, C).max(axis=(2, 4))


def maxpool2_bwd(a: np.ndarray, dout: np.ndarray) -> np.ndarray:
    """MaxPoolGrad: each window's gradient goes to its FIRST maximum in row-major scan order
    (TF CPU MaxPool argmax semantics; ties only occur between zeros after ReLU, whose
    gradient the following ReLU mask removes)."""
    N, H, W, C = a.shape
    w4 = a.reshape(N, H // 2, 2, W // 2, 2, C).transpose(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, C)
    arg = w4.argmax(axis=3)  # numpy argmax returns the first maximum
    g4 = np.zeros_like(w4)
    np.put_along_axis(g4, arg[:, :, :, None, :], dout[:, :, :, None, :], axis=3)
    return g4.reshape(N, H // 2, W // 2, 2, 2, C).transpose(0, 1, 3, 2, 4, 5).reshape(N, H, W, C)


# ------------------------------------------------------------------- Conv2DTranspose -----
def conv_transpose2x2(x: np.ndarray, k: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Conv2DTranspose(f, 2, strides=2, padding='same') (model/u_net.py:88-94):
    out[n,2i+a,2j+b,co] = sum_ci x[n,i,j,ci] k[a,b,co,ci] + bias[co] (no overlap, no flip)."""
    N, H, W, Ci = x.shape
    f = k.shape[2]
    o = np.einsum("nijc,abdc->niajbd", x, k)
    return o.reshape(N, 2 * H, 2 * W, f) + b


def conv_transpose2x2_bwd(x, k, dout):
    N, H, W, Ci = x.shape
    f = k.shape[2]
    d6 = dout.reshape(N, H, 2, W, 2, f)
    dx = np.einsum("niajbd,abdc->nijc", d6, k)
    dk = np.einsum("niajbd,nijc->abdc", d6, x)
    db = dout.reshape(-1, f).sum(axis=0)
    return dx, dk, db


# ------------------------------------------------------------------------ output head ----
def head(x, k, b, num_classes):
    """Conv2D(ncls, 1, padding='same', activation=sigmoid|softmax) (model/u_net.py:105-112)."""
    logits = pointwise(x, k) + b
    if num_classes == 1:
        return 1.0 / (1.0 + np.exp(-logits))
    e = np.exp(logits - logits.max(axis=-1, keepdims=True))
    return e / e.sum(axis=-1, keepdims=True)


def head_bwd(x, k, prob, dprob, num_classes):
    if num_classes == 1:
        dl = dprob * prob * (1 - prob)
    else:
        dl = prob * (dprob - (dprob * prob).sum(axis=-1, keepdims=True))
    dx, dk = pointwise_bwd(x, k, dl)
    db = dl.reshape(-1, dl.shape[-1]).sum(axis=0)
    return dx, dk, db


# ------------------------------------------------------------------ losses / metrics -----
def dice_sums(y_true, y_pred):
    """Per (batch, channel) sums over H,W (utils/metrics.py:26-30)."""
    i = (y_true * y_pred).sum(axis=(1, 2))
    t = y_true.sum(axis=(1, 2))
    p = y_pred.sum(axis=(1, 2))
    return i, t, p


def dice_coef(y_true, y_pred, smooth=SMOOTH):
    """utils/metrics.py:6-39: mean over (batch, channel) of (2I + s) / (T + P + s)."""
    i, t, p = dice_sums(y_true, y_pred)
    return ((2.0 * i + smooth) / (t + p + smooth)).mean()


def iou_coef(y_true, y_pred, smooth=SMOOTH):
    """utils/metrics.py:41-62: mean of (I + s) / (T + P - I + s)."""
    i, t, p = dice_sums(y_true, y_pred)
    return ((i + smooth) / (t + p - i + smooth)).mean()


def dice_loss(y_true, y_pred):
    """utils/loss.py:9-29: 1 - dice_coef."""
    return 1.0 - dice_coef(y_true, y_pred)


def iou_loss(y_true, y_pred, smooth=SMOOTH):
    """utils/loss.py:31-45 (intended semantics; the reference forgets to import iou_coef)."""
    return 1.0 - iou_coef(y_true, y_pred, smooth)


def dice_loss_grad(y_true, y_pred, smooth=SMOOTH):
    i, t, p = dice_sums(y_true, y_pred)
    nm = 2 * i + smooth
    den = t + p + smooth
    B, C = i.shape
    return -(2 * y_true * den[:, None, None, :] - nm[:, None, None, :]) / (den[:, None, None, :] ** 2) / (B * C)


def iou_loss_grad(y_true, y_pred, smooth=SMOOTH):
    i, t, p = dice_sums(y_true, y_pred)
    j = (i + smooth)[:, None, None, :]
    u = (t + p - i + smooth)[:, None, None, :]
    B, C = i.shape
    return -(y_true * u - j * (1 - y_true)) / (u ** 2) / (B * C)


def meaniou_confusion(y_true, y_pred, num_classes, threshold=None):
    """keras.metrics.MeanIoU.update_state (scripts/train.py:231, benchmark.py:269): labels and
    predictions cast float -> int64 (truncation) unless thresholded first (benchmark.py:260);
    confusion[true][pred] counts; out-of-range labels skipped."""
    t = np.trunc(np.asarray(y_true, dtype=np.float64).ravel()).astype(np.int64)
    yp = np.asarray(y_pred, dtype=np.float64).ravel()
    if threshold is None:
        p = np.trunc(yp).astype(np.int64)
    else:
        p = (yp > threshold).astype(np.int64)
    ok = (t >= 0) & (t < num_classes) & (p >= 0) & (p < num_classes)
    cm = np.zeros((num_classes, num_classes), dtype=np.int64)
    np.add.at(cm, (t[ok], p[ok]), 1)
    return cm


def meaniou_result(cm):
    """MeanIoU.result(): IoU_k = cm_kk / (row_k + col_k - cm_kk); mean over classes whose
    denominator is nonzero (divide_no_nan semantics)."""
    cm = cm.astype(np.float64)
    tp = np.diag(cm)
    den = cm.sum(axis=0) + cm.sum(axis=1) - tp
    valid = den != 0
    if not valid.any():
        return 0.0
    return float((tp[valid] / den[valid]).sum() / valid.sum())


# ----------------------------------------------------------------------------- AdamW -----
def adamw_update(p, g, m, v, step, lr, wd, beta1=0.9, beta2=0.999, eps=1e-7):
    """keras.optimizers.AdamW (scripts/train.py:226), Keras 3 update order: weight decay
    first (p -= p*wd*lr), then m, v, and p -= m*alpha/(sqrt(v)+eps) with
    alpha = lr*sqrt(1-b2^t)/(1-b1^t), t = step (1-based).  Returns new (p, m, v)."""
    p = p - p * wd * lr
    m = m + (g - m) * (1 - beta1)
    v = v + (g * g - v) * (1 - beta2)
    alpha = lr * np.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    p = p - (m * alpha) / (np.sqrt(v) + eps)
    return p, m, v
