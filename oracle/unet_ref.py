"""CPU oracle: the whole U-Net of the reference (model/u_net.py:28-116) as NumPy, forward,
backward (GradientTape of scripts/train.py:308 `model.fit`), and one AdamW train step.

TEST INFRASTRUCTURE ONLY (see oracle/keras_ops.py header).  PARITY UNPINNED by the
reference itself: it has no tests or golden data and TensorFlow is not importable here.

Parameters are a dict keyed by the reference's Keras weight names
("enc1_block1_sepconv/depthwise_kernel", "enc1_block1_bn/gamma", "dec4_upsample/kernel",
"output_mask/bias", ...) in Keras layouts.
"""
from __future__ import annotations

import numpy as np

from . import keras_ops as K

FILTERS = (64, 128, 256, 512)  # model/u_net.py:57


def _stages(filters):
    enc = [(f"enc{i + 1}", f) for i, f in enumerate(filters)]
    dec = [(f"dec{len(filters) - i}", f) for i, f in enumerate(reversed(filters))]
    return enc, dec


class UNetOracle:
    def __init__(self, num_classes=1, dropout_rate=0.2, use_batch_norm=True, filters=FILTERS):
        self.num_classes = num_classes
        self.dropout_rate = dropout_rate
        self.use_bn = use_batch_norm
        self.filters = tuple(filters)

    # ---------------------------------------------------------------- conv_block ------
    def _block_fwd(self, p, name, a, training, cache, new_stats):
        """conv_block (model/u_net.py:5-26): SeparableConv2D -> [BatchNormalization] -> ReLU."""
        dk = p[f"{name}_sepconv/depthwise_kernel"]
        pk = p[f"{name}_sepconv/pointwise_kernel"]
        y = K.depthwise3x3(a, dk)
        z = K.pointwise(y, pk)
        rec = {"a_in": a, "y": y, "z": z}
        if self.use_bn:
            g, b = p[f"{name}_bn/gamma"], p[f"{name}_bn/beta"]
            if training:
                out, mean, var = K.bn_train(z, g, b)
                mm, mv = K.bn_moving_update(p[f"{name}_bn/moving_mean"], p[f"{name}_bn/moving_variance"], mean, var)
                new_stats[f"{name}_bn/moving_mean"] = mm
                new_stats[f"{name}_bn/moving_variance"] = mv
                rec.update(mean=mean, var=var)
            else:
                out = K.bn_infer(z, g, b, p[f"{name}_bn/moving_mean"], p[f"{name}_bn/moving_variance"])
        else:
            out = z + p[f"{name}_sepconv/bias"]
        cache[name] = rec
        return K.relu(out)

    def _block_bwd(self, p, name, da, cache, grads, drop=None):
        rec = cache[name]
        dk = p[f"{name}_sepconv/depthwise_kernel"]
        pk = p[f"{name}_sepconv/pointwise_kernel"]
        if self.use_bn:
            dz, dgamma, dbeta = K.bn_relu_bwd(da, rec["z"], p[f"{name}_bn/gamma"], p[f"{name}_bn/beta"],
                                              rec["mean"], rec["var"], drop=drop)
            grads[f"{name}_bn/gamma"] = dgamma
            grads[f"{name}_bn/beta"] = dbeta
        else:
            pre = rec["z"] + p[f"{name}_sepconv/bias"]
            g = da if drop is None else da * drop
            dz = np.where(pre > 0, g, 0)
            grads[f"{name}_sepconv/bias"] = dz.reshape(-1, dz.shape[-1]).sum(axis=0)
        dy, dpk = K.pointwise_bwd(rec["y"], pk, dz)
        da_in, ddk = K.depthwise3x3_bwd(rec["a_in"], dk, dy)
        grads[f"{name}_sepconv/pointwise_kernel"] = dpk
        grads[f"{name}_sepconv/depthwise_kernel"] = ddk
        return da_in

    # ------------------------------------------------------------------- forward ------
    def forward(self, p, x, training=False, drop_seeds=None):
        """U_NET forward (model/u_net.py:55-112).  Returns (prob, cache, new_moving_stats)."""
        cache, new_stats = {}, {}
        enc, dec = _stages(self.filters)
        drop_on = training and self.dropout_rate > 0.0
        a = x
        skips = []
        for stage, f in enc:
            a = self._block_fwd(p, f"{stage}_block1", a, training, cache, new_stats)
            a = self._block_fwd(p, f"{stage}_block2", a, training, cache, new_stats)
            skips.append(a)
            cache[f"{stage}_skip"] = a
            a = K.maxpool2(a)
        a = self._block_fwd(p, "bneck_block1", a, training, cache, new_stats)
        a = self._block_fwd(p, "bneck_block2", a, training, cache, new_stats)
        if drop_on:
            m = K.dropout_mult(drop_seeds["bneck_dropout"], a.shape, self.dropout_rate, a.dtype)
            cache["bneck_dropmask"] = m
            a = a * m
        for i, (stage, f) in enumerate(dec):
            x_in = a
            u = K.conv_transpose2x2(x_in, p[f"{stage}_upsample/kernel"], p[f"{stage}_upsample/bias"])
            cat = np.concatenate([u, skips[len(skips) - 1 - i]], axis=-1)  # [x, skip] (u_net.py:96)
            if drop_on and i < len(dec) - 1:
                m = K.dropout_mult(drop_seeds[f"{stage}_dropout"], cat.shape, self.dropout_rate, cat.dtype)
                cache[f"{stage}_dropmask"] = m
                cat = cat * m
            cache[f"{stage}_upsample"] = {"x": x_in, "f": f}
            a = self._block_fwd(p, f"{stage}_block1", cat, training, cache, new_stats)
            a = self._block_fwd(p, f"{stage}_block2", a, training, cache, new_stats)
        cache["head_x"] = a
        prob = K.head(a, p["output_mask/kernel"], p["output_mask/bias"], self.num_classes)
        cache["prob"] = prob
        return prob, cache, new_stats

    # ------------------------------------------------------------------ backward ------
    def backward(self, p, cache, dprob, trace=None):
        """Gradients of every trainable variable given dL/dprob.  If `trace` is a dict it
        receives the gradient w.r.t. each conv_block's output activation, keyed by block."""
        grads = {}
        if trace is not None:
            _bb = self._block_bwd

            def _traced(p_, name, da, cache_, grads_, drop=None):
                trace[name] = da
                return _bb(p_, name, da, cache_, grads_, drop)
            self._block_bwd = _traced
        enc, dec = _stages(self.filters)
        da, dkh, dbh = K.head_bwd(cache["head_x"], p["output_mask/kernel"], cache["prob"], dprob, self.num_classes)
        grads["output_mask/kernel"] = dkh
        grads["output_mask/bias"] = dbh
        dskips = {}
        for i in reversed(range(len(dec))):
            stage, f = dec[i]
            da = self._block_bwd(p, f"{stage}_block2", da, cache, grads)
            dcat = self._block_bwd(p, f"{stage}_block1", da, cache, grads)
            if f"{stage}_dropmask" in cache:
                dcat = dcat * cache[f"{stage}_dropmask"]
            du, dskip = dcat[..., :f], dcat[..., f:]
            enc_stage = enc[len(enc) - 1 - i][0]
            dskips[enc_stage] = dskip
            rec = cache[f"{stage}_upsample"]
            da, dk, db = K.conv_transpose2x2_bwd(rec["x"], p[f"{stage}_upsample/kernel"], du)
            grads[f"{stage}_upsample/kernel"] = dk
            grads[f"{stage}_upsample/bias"] = db
        drop = cache.get("bneck_dropmask")
        da = self._block_bwd(p, "bneck_block2", da, cache, grads, drop=drop)
        da = self._block_bwd(p, "bneck_block1", da, cache, grads)
        for stage, f in reversed(enc):
            skip_a = cache[f"{stage}_skip"]
            da = dskips[stage] + K.maxpool2_bwd(skip_a, da)
            da = self._block_bwd(p, f"{stage}_block2", da, cache, grads)
            da = self._block_bwd(p, f"{stage}_block1", da, cache, grads)
        if trace is not None:
            del self._block_bwd
        return grads, da

    # ---------------------------------------------------------------- train step ------
    def loss_and_dprob(self, y_true, prob, loss="dice"):
        if loss == "dice":
            return K.dice_loss(y_true, prob), K.dice_loss_grad(y_true, prob)
        return K.iou_loss(y_true, prob), K.iou_loss_grad(y_true, prob)

    def train_step(self, p, opt, x, y_true, step, lr, wd, drop_seeds=None, loss="dice"):
        """One Keras `train_step` (scripts/train.py:308): forward(training=True), loss,
        backward, AdamW over every trainable variable, moving-stat update.  `opt` maps name ->
        (m, v); `step` is the 1-based iteration.  Returns (loss, dice, grads, new_params, new_opt)."""
        prob, cache, new_stats = self.forward(p, x, training=True, drop_seeds=drop_seeds)
        lval, dprob = self.loss_and_dprob(y_true, prob, loss)
        grads, _ = self.backward(p, cache, dprob)
        newp = dict(p)
        newo = {}
        for name, g in grads.items():
            m, v = opt[name]
            newp[name], m2, v2 = K.adamw_update(p[name], g, m, v, step, lr, wd)
            newo[name] = (m2, v2)
        newp.update(new_stats)
        return lval, K.dice_coef(y_true, prob), grads, newp, newo, prob
