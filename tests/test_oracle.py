"""The oracle against an independent restatement: torch-CPU float64 autograd of the same
graph (torch.nn.functional convs with Keras layouts permuted to torch's).  This checks the
oracle's hand-derived backward, its layouts and its op conventions; the reference itself
cannot run here (TensorFlow absent), so parity with TF stays unpinned."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import keras_ops as K
from oracle.unet_ref import UNetOracle
from unet_amd.params import init_weights, unet_variables


def _torch_unet(p, x, ncls, use_bn, filters, masks, training=True):
    t = {k: torch.tensor(v, dtype=torch.float64, requires_grad="moving" not in k) for k, v in p.items()}
    h = torch.tensor(x).permute(0, 3, 1, 2)

    def block(a, name):
        dk, pk = t[f"{name}_sepconv/depthwise_kernel"], t[f"{name}_sepconv/pointwise_kernel"]
        y = F.conv2d(a, dk.permute(2, 3, 0, 1), padding=1, groups=a.shape[1])
        z = F.conv2d(y, pk.permute(3, 2, 0, 1))
        if use_bn:
            if training:
                z = F.batch_norm(z, None, None, t[f"{name}_bn/gamma"], t[f"{name}_bn/beta"], True, 0.0, 1e-3)
            else:
                z = F.batch_norm(z, t[f"{name}_bn/moving_mean"], t[f"{name}_bn/moving_variance"],
                                 t[f"{name}_bn/gamma"], t[f"{name}_bn/beta"], False, 0.0, 1e-3)
        else:
            z = z + t[f"{name}_sepconv/bias"][None, :, None, None]
        return F.relu(z)

    skips = []
    for i in range(len(filters)):
        h = block(h, f"enc{i + 1}_block1")
        h = block(h, f"enc{i + 1}_block2")
        skips.append(h)
        h = F.max_pool2d(h, 2)
    h = block(h, "bneck_block1")
    h = block(h, "bneck_block2")
    if "bneck_dropout" in masks:
        h = h * torch.tensor(masks["bneck_dropout"]).permute(0, 3, 1, 2)
    for i in range(len(filters)):
        st = f"dec{len(filters) - i}"
        u = F.conv_transpose2d(h, t[f"{st}_upsample/kernel"].permute(3, 2, 0, 1), t[f"{st}_upsample/bias"], stride=2)
        h = torch.cat([u, skips[len(filters) - 1 - i]], 1)
        if f"{st}_dropout" in masks:
            h = h * torch.tensor(masks[f"{st}_dropout"]).permute(0, 3, 1, 2)
        h = block(h, f"{st}_block1")
        h = block(h, f"{st}_block2")
    logits = F.conv2d(h, t["output_mask/kernel"].permute(3, 2, 0, 1), t["output_mask/bias"])
    prob = torch.sigmoid(logits) if ncls == 1 else torch.softmax(logits, 1)
    return prob.permute(0, 2, 3, 1), t


def _dice_loss_t(y, p):
    i = (y * p).sum((1, 2))
    d = (2 * i + 1e-7) / (y.sum((1, 2)) + p.sum((1, 2)) + 1e-7)
    return 1 - d.mean()


@pytest.mark.parametrize("ncls,use_bn,drop,hw,filters", [(1, True, 0.0, 32, (8, 16, 32, 64)),
                                                        (1, True, 0.3, 32, (8, 16, 32, 64)),
                                                        (5, True, 0.0, 16, (8, 16, 32, 64)),
                                                        (1, False, 0.0, 16, (4, 8, 8, 16)),
                                                        (1, True, 0.0, 16, (64, 128, 256, 512))])
def test_oracle_matches_torch_autograd(ncls, use_bn, drop, hw, filters):
    rng = np.random.default_rng(ncls + hw)
    specs = unet_variables(3, ncls, use_bn, filters)
    p = {k: v.astype(np.float64) for k, v in init_weights(specs, 7).items()}
    x = rng.random((2, hw, hw, 3))
    y = (rng.random((2, hw, hw, ncls)) > 0.5).astype(np.float64)
    orc = UNetOracle(ncls, drop, use_bn, filters)
    seeds = {s: 100 + i for i, s in enumerate(("bneck_dropout", "dec4_dropout", "dec3_dropout", "dec2_dropout"))}
    prob, cache, _ = orc.forward(p, x, training=True, drop_seeds=seeds)
    loss, dprob = orc.loss_and_dprob(y, prob)
    grads, dx = orc.backward(p, cache, dprob)
    masks = {k[:-len("dropmask")] + "dropout": v for k, v in cache.items() if k.endswith("dropmask")}
    assert len(masks) == (4 if drop > 0 else 0)
    tp, tt = _torch_unet(p, x, ncls, use_bn, filters, masks)
    tl = _dice_loss_t(torch.tensor(y), tp)
    tl.backward()
    assert np.abs(tp.detach().numpy() - prob).max() < 1e-12
    assert abs(tl.item() - loss) < 1e-12
    for k, g in grads.items():
        ref = tt[k].grad.numpy()
        assert np.abs(g - ref).max() <= 1e-9 * (np.abs(ref).max() + 1e-12), k
    assert set(grads) == {k for k, v in tt.items() if v.grad is not None}


def test_oracle_inference_matches_torch():
    specs = unet_variables(3, 1, True, (8, 16, 16, 32))
    rng = np.random.default_rng(1)
    p = {k: v.astype(np.float64) for k, v in init_weights(specs, 3).items()}
    for k in p:
        if k.endswith("moving_mean"):
            p[k] = rng.standard_normal(p[k].shape) * 0.1
        if k.endswith("moving_variance"):
            p[k] = 0.5 + rng.random(p[k].shape)
    x = rng.random((2, 32, 32, 3))
    prob, _, _ = UNetOracle(1, 0.2, True, (8, 16, 16, 32)).forward(p, x, training=False)
    tp, _ = _torch_unet(p, x, 1, True, (8, 16, 16, 32), {}, training=False)
    assert np.abs(tp.detach().numpy() - prob).max() < 1e-12


def test_maxpool_first_max_routing():
    a = np.zeros((1, 2, 2, 2))
    a[0, 0, 1, 0] = a[0, 1, 0, 0] = 3.0  # tie between (0,1) and (1,0): first in scan order wins
    a[0, 1, 1, 1] = 1.0
    g = K.maxpool2_bwd(a, np.ones((1, 1, 1, 2)))
    assert g[0, 0, 1, 0] == 1 and g[0, 1, 0, 0] == 0 and g[0, 1, 1, 1] == 1


def test_dropout_mask_statistics():
    m = K.dropout_mult(12345, (4, 64, 64, 32), 0.2, np.float64)
    keep = (m > 0).mean()
    assert abs(keep - 0.8) < 0.005
    assert np.allclose(m[m > 0], 1 / np.float32(0.8))
    assert not np.array_equal(m, K.dropout_mult(12346, m.shape, 0.2))


def test_adamw_keras_epsilon_placement():
    p, g = np.array([1.0]), np.array([0.5])
    p1, m1, v1 = K.adamw_update(p, g, np.zeros(1), np.zeros(1), 1, 1e-3, 0.0)
    # first step: m = 0.1 g, v = 0.001 g^2, alpha = lr*sqrt(0.001)/0.1 -> step = lr*g/(|g| + eps/sqrt(.001))
    expect = 1.0 - 1e-3 * 0.5 / (0.5 + 1e-7 / np.sqrt(1e-3))
    assert abs(p1[0] - expect) < 1e-15


def test_meaniou_semantics():
    yt = np.array([0, 1, 1, 0, 1.0])
    yp = np.array([0.2, 0.999, 1.0, 0.7, 0.6])
    cm = K.meaniou_confusion(yt, yp, 2)  # truncation: only p == 1.0 counts as class 1
    assert cm.tolist() == [[2, 0], [2, 1]]
    cm2 = K.meaniou_confusion(yt, yp, 2, 0.5)
    assert cm2.tolist() == [[1, 1], [0, 3]]
    assert abs(K.meaniou_result(cm2) - (1 / 2 + 3 / 4) / 2) < 1e-15
