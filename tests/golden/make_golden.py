"""Generates tests/golden/*.npz from the NumPy oracle (oracle/).  Inputs and weights come from
the portable splitmix64 stream (unet_amd.params.portable_uniform), so every vector here can be
regenerated bit-for-bit; outputs are float64 oracle results stored as float32/float64.

The reference itself ships no golden data and cannot run here (TensorFlow absent), so these
fixtures freeze the oracle (parity unpinned against TF), they do not pin it.

    python tests/golden/make_golden.py [fixture.npz ...]

The BASELINE-size fixtures (fwd256/fwd512/fwd21/samples/train128) hold the configs[1], [3] and
[4] geometries at inference and one train step at 128x128 batch 4; samples/ holds the two
images of the reference's samples/test_images (input data) and, under samples/usage, the
reference's own inference outputs for them (samples/usage/*: output_mask.png,
output_cropped.png), which pin the post-processing crop (tests/test_imageproc.py).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]

from oracle import keras_ops as K  # noqa: E402
from oracle.unet_ref import UNetOracle  # noqa: E402
from unet_amd.params import init_weights, portable_uniform, unet_variables  # noqa: E402


def U(seed, shape, lo=0.0, hi=1.0):
    n = int(np.prod(shape))
    return (lo + (hi - lo) * portable_uniform(seed, n)).reshape(shape).astype(np.float32).astype(np.float64)


def model_weights(ncls, filters, seed):
    specs = unet_variables(3, ncls, True, filters)
    w = {k: v.astype(np.float64) for k, v in init_weights(specs, seed).items()}
    for i, k in enumerate(sorted(w)):
        if k.endswith("moving_mean"):
            w[k] = U(seed + 100 + i, w[k].shape, -0.2, 0.2)
        elif k.endswith("moving_variance"):
            w[k] = U(seed + 100 + i, w[k].shape, 0.5, 1.5)
        elif k.endswith("gamma"):
            w[k] = U(seed + 100 + i, w[k].shape, 0.7, 1.3)
        elif k.endswith("beta"):
            w[k] = U(seed + 100 + i, w[k].shape, -0.1, 0.1)
    return w


def ops_fixture():
    out = {}
    x = U(1, (2, 8, 8, 16), -1, 1)
    dk = U(2, (3, 3, 16, 1), -1, 1)
    dy = U(3, (2, 8, 8, 16), -1, 1)
    out.update(dw_x=x, dw_k=dk, dw_dy=dy, dw_y=K.depthwise3x3(x, dk))
    out["dw_dx"], out["dw_dk"] = K.depthwise3x3_bwd(x, dk, dy)
    pk = U(4, (1, 1, 16, 32), -0.3, 0.3)
    z = K.pointwise(x, pk)
    dz = U(5, z.shape, -1, 1)
    out.update(pw_k=pk, pw_z=z, pw_dz=dz)
    out["pw_dx"], out["pw_dk"] = K.pointwise_bwd(x, pk, dz)
    gamma, beta = U(6, (32,), 0.5, 1.5), U(7, (32,), -0.2, 0.2)
    bn_out, mean, var = K.bn_train(z, gamma, beta)
    da = U(8, z.shape, -1, 1)
    out.update(bn_gamma=gamma, bn_beta=beta, bn_out=bn_out, bn_mean=mean, bn_var=var, bn_da=da)
    out["bn_dz"], out["bn_dgamma"], out["bn_dbeta"] = K.bn_relu_bwd(da, z, gamma, beta, mean, var)
    a = K.relu(bn_out)
    out["pool_out"] = K.maxpool2(a)
    out["pool_dx"] = K.maxpool2_bwd(a, U(9, out["pool_out"].shape, -1, 1))
    out["pool_dout"] = U(9, out["pool_out"].shape, -1, 1)
    ck, cb = U(10, (2, 2, 8, 16), -0.3, 0.3), U(11, (8,), -0.1, 0.1)
    co = K.conv_transpose2x2(x, ck, cb)
    cdo = U(12, co.shape, -1, 1)
    out.update(ct_k=ck, ct_b=cb, ct_out=co, ct_dout=cdo)
    out["ct_dx"], out["ct_dk"], out["ct_db"] = K.conv_transpose2x2_bwd(x, ck, cdo)
    yt = (U(13, (2, 8, 8, 1)) > 0.5).astype(np.float64)
    yp = U(14, (2, 8, 8, 1))
    out.update(dice_yt=yt, dice_yp=yp, dice_loss=K.dice_loss(yt, yp), dice_coef=K.dice_coef(yt, yp),
               iou_coef=K.iou_coef(yt, yp), dice_grad=K.dice_loss_grad(yt, yp))
    out["miou_cm_trunc"] = K.meaniou_confusion(yt, yp, 2)
    out["miou_cm_thr"] = K.meaniou_confusion(yt, yp, 2, 0.5)
    p, g, m, v = U(15, (100,), -1, 1), U(16, (100,), -0.1, 0.1), U(17, (100,), -0.01, 0.01), U(18, (100,), 0, 0.01)
    out.update(adam_p=p, adam_g=g, adam_m=m, adam_v=v)
    out["adam_p1"], out["adam_m1"], out["adam_v1"] = K.adamw_update(p, g, m, v, 3, 2e-3, 1e-4)
    out["drop_mask"] = K.dropout_mult(2301, (2, 4, 4, 8), 0.2)
    return out


def cfg1_fixture():
    """configs[0]: U_NET((128,128,3), 1) forward on 2 images (inference mode)."""
    w = model_weights(1, (64, 128, 256, 512), 2301)
    x = U(7, (2, 128, 128, 3))
    prob, _, _ = UNetOracle(1).forward(w, x, training=False)
    return {"x_seed": 7, "w_seed": 2301, "prob": prob.astype(np.float32)}


def train_fixture():
    """One train step (dropout 0) at 32x32, batch 2, full widths: loss, dice, per-tensor grad
    norms, and post-AdamW values of a few tensors."""
    w = model_weights(1, (64, 128, 256, 512), 11)
    x = U(21, (2, 32, 32, 3))
    y = (U(22, (2, 32, 32, 1)) > 0.6).astype(np.float64)
    orc = UNetOracle(1, 0.0)
    opt = {k: (np.zeros_like(v), np.zeros_like(v)) for k, v in w.items() if "moving" not in k}
    loss, dice, g, newp, _, prob = orc.train_step(w, opt, x, y, 1, 2e-3, 1e-4)
    out = {"x_seed": 21, "y_seed": 22, "w_seed": 11, "loss": loss, "dice": dice}
    for k, v in g.items():
        out["gnorm:" + k] = np.linalg.norm(v)
    for k in ("output_mask/kernel", "dec1_block2_bn/gamma", "enc1_block1_sepconv/pointwise_kernel"):
        out["new:" + k] = newp[k]
    return out


FULL = (64, 128, 256, 512)


def quad_masks(n, h, w, ncls=1):
    """Deterministic ID-card-like axis-aligned quads (about 30 % foreground) per image."""
    y = np.zeros((n, h, w, 1), np.float64)
    for i in range(n):
        u = portable_uniform(900 + i, 4)
        hh, ww = int(h * (0.4 + 0.3 * u[0])), int(w * (0.4 + 0.3 * u[1]))
        y0, x0 = int(u[2] * (h - hh)), int(u[3] * (w - ww))
        y[i, y0:y0 + hh, x0:x0 + ww] = 1.0
    return y


def fwd256_fixture():
    """configs[1] geometry (256x256x3, binary) inference forward on 2 images."""
    w = model_weights(1, FULL, 2301)
    x = U(31, (2, 256, 256, 3))
    prob, _, _ = UNetOracle(1).forward(w, x, training=False)
    return {"x_seed": 31, "w_seed": 2301, "prob": prob.astype(np.float32)}


def fwd512_fixture():
    """configs[3] geometry (512x512x3, binary) inference forward on 1 image."""
    w = model_weights(1, FULL, 2301)
    x = U(32, (1, 512, 512, 3))
    prob, _, _ = UNetOracle(1).forward(w, x, training=False)
    return {"x_seed": 32, "w_seed": 2301, "prob": prob.astype(np.float32)}


def fwd21_fixture():
    """configs[4] geometry (256x256x3, 21 classes, softmax head) inference forward on 2 images:
    probabilities on every 4th pixel, the full argmax map and per-(image, class) sums."""
    w = model_weights(21, FULL, 2302)
    x = U(33, (2, 256, 256, 3))
    prob, _, _ = UNetOracle(21).forward(w, x, training=False)
    return {"x_seed": 33, "w_seed": 2302, "prob_s4": prob[:, ::4, ::4, :].astype(np.float32),
            "argmax": prob.argmax(-1).astype(np.uint8), "class_sums": prob.sum((1, 2))}


def samples_fixture():
    """The reference's samples/test_images/*.png through the inference preprocessing
    (scripts/inference.py:98-110: BGR, /255, INTER_LINEAR to 256x256; restated in
    scripts/inference.py here) and the forward of the 2301-seeded weights."""
    sys.path.insert(0, os.path.join(ROOT, "unet-image-segmentation_amd", "scripts"))
    import inference  # the drop-in CLI module (its preprocessing)
    w = model_weights(1, FULL, 2301)
    out = {"w_seed": 2301}
    for name in SAMPLE_NAMES:
        x, bgr, h, wd = inference.load_and_preprocess_image(os.path.join(HERE, "samples", name + ".png"), 256, 256)
        prob, _, _ = UNetOracle(1).forward(w, x.astype(np.float64), training=False)
        out[name + ":x_sum"] = float(x.astype(np.float64).sum())
        out[name + ":x_s8"] = x[:, ::8, ::8, :]
        out[name + ":prob"] = prob.astype(np.float32)
    return out


SAMPLE_NAMES = ("brazil_passport", "chile_id_card")


def train128_fixture():
    """One train step (dropout 0) at 128x128, batch 4, full widths: loss, dice, every gradient's
    norm and first 128 values, the first 256 post-AdamW values and moving statistics of every
    variable."""
    w = model_weights(1, FULL, 11)
    x = U(41, (4, 128, 128, 3))
    y = quad_masks(4, 128, 128)
    orc = UNetOracle(1, 0.0)
    opt = {k: (np.zeros_like(v), np.zeros_like(v)) for k, v in w.items() if "moving" not in k}
    loss, dice, g, newp, _, prob = orc.train_step(w, opt, x, y, 1, 2e-3, 1e-4)
    out = {"x_seed": 41, "w_seed": 11, "loss": loss, "dice": dice}
    for k, v in g.items():
        out["gnorm:" + k] = np.linalg.norm(v)
        out["g128:" + k] = v.reshape(-1)[:128]
    for k, v in newp.items():
        out["new256:" + k] = v.reshape(-1)[:256]
    return out


SUB = 16384  # gradient elements kept per tensor in the training-geometry fixtures
SUB_STRIDE = 1000003  # prime: coprime to every gradient size (2^a * 3^b * 7^c, all < 2^22)


def sub_index(size):
    """Deterministic subsample of a flat tensor (all of it when it is small): i * P mod size for
    i < SUB with P prime, sorted.  P is odd, so i -> i * P is a bijection mod every power of two:
    the SUB consecutive i hit every residue of the flat index mod 2^k equally often for
    2^k <= SUB, i.e. every output channel (the innermost Keras axis, <= 1024) of a pointwise /
    Conv2DTranspose kernel gets SUB / Cout samples, spread over the input-channel axis too.
    (Rounds 3-4 used the stride size // SUB, which for a 512 x 1024 kernel sampled only output
    channels 0, 32, ..., 992 -- lane 0 of every 32-column MFMA tile)"""
    if size <= SUB:
        return np.arange(size)
    assert np.gcd(size, SUB_STRIDE) == 1, size
    return np.sort((np.arange(SUB, dtype=np.int64) * SUB_STRIDE) % size)


def channel_norms(v):
    """Per-output-channel and per-input-channel L2 norms of a Keras-layout gradient: the last axis
    (pointwise / head: Cout; depthwise: the multiplier 1; Conv2DTranspose: Cin) and the second to
    last (pointwise: Cin; depthwise: C; Conv2DTranspose: its filters f).  Vectors: |v| itself."""
    v = np.asarray(v, np.float64)
    if v.ndim < 2:
        a = np.abs(v).reshape(-1)
        return a, a
    last = np.sqrt((v.reshape(-1, v.shape[-1]) ** 2).sum(0))
    sec = np.sqrt((np.moveaxis(v, -2, -1).reshape(-1, v.shape[-2]) ** 2).sum(0))
    return last, sec


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64).reshape(-1), np.asarray(b, np.float64).reshape(-1)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def class_masks(n, h, w, ncls, seed):
    """One-hot class maps for the multi-class geometry: 8x8-pixel cells of uniformly drawn classes."""
    cells = np.floor(U(seed, (n, h // 8, w // 8)) * ncls).astype(np.int64).clip(0, ncls - 1)
    cls = cells.repeat(8, 1).repeat(8, 2)
    return np.eye(ncls)[cls]


DROP_SITES = ("bneck_dropout", "dec4_dropout", "dec3_dropout", "dec2_dropout")


def _mix64(*vals):
    """The engine's dropout-seed mixer (unet_amd/engine.py _mix64), restated so the fixture does not
    need the device library: splitmix64 finalisers folded over the values."""
    z = 0x243F6A8885A308D3
    M = 0xFFFFFFFFFFFFFFFF
    for v in vals:
        z = (z ^ (int(v) & M)) & M
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
    return z


def engine_drop_seeds(seed, step):
    """Per-site dropout seeds of a single-process engine step (UNetEngine.drop_seeds, rank_salt 0):
    the GPU test checks the engine still draws exactly these before comparing."""
    return {s: _mix64(seed, step, i + 1) for i, s in enumerate(DROP_SITES)}


def train_big_fixture(size, n, ncls, x_seed, w_seed, drop=0.0, engine_seed=2301):
    """One train step at a BASELINE training geometry, full widths, float64 oracle (dropout off,
    or `drop` = the reference's default 0.2 with the engine's first-step masks):
    loss, dice, every block's BatchNorm batch mean / variance, every gradient's norm, first 128
    values and a strided subsample (sub_index) with e32 = the same step in float32 (its own
    relative-L2 distance to float64 on that subsample, and over the whole tensor), and the first
    256 post-AdamW values of every variable (moving statistics included).  Too slow to run live on
    the GPU box (about 4 minutes at 256x256 x 16 here), so the box only compares."""
    w = model_weights(ncls, FULL, w_seed)
    x = U(x_seed, (n, size, size, 3))
    y = quad_masks(n, size, size) if ncls == 1 else class_masks(n, size, size, ncls, x_seed + 1)
    orc = UNetOracle(ncls, drop)
    seeds = engine_drop_seeds(engine_seed, 1) if drop > 0 else None
    out = {"x_seed": x_seed, "w_seed": w_seed, "n": n, "size": size, "ncls": ncls, "drop": drop,
           "engine_seed": engine_seed}
    if seeds:
        for k, v in seeds.items():
            out["drop_seed:" + k] = np.uint64(v)
    prob, cache, stats = orc.forward(w, x, training=True, drop_seeds=seeds)
    lval, dprob = orc.loss_and_dprob(y, prob)
    out["loss"], out["dice"] = lval, K.dice_coef(y, prob)
    for name, rec in cache.items():
        if isinstance(rec, dict) and "mean" in rec:
            out["bn_mean:" + name], out["bn_var:" + name] = rec["mean"], rec["var"]
    del prob
    g, _ = orc.backward(w, cache, dprob)
    del cache, dprob
    for k, v in g.items():
        flat = v.reshape(-1)
        out["gnorm:" + k] = np.linalg.norm(flat)
        out["g128:" + k] = flat[:128]
        out["gsub:" + k] = flat[sub_index(flat.size)].astype(np.float32)
        out["cn_last:" + k], out["cn_sec:" + k] = channel_norms(v)
    for k, v in w.items():
        if k in g:
            p1, _, _ = K.adamw_update(v, g[k], np.zeros_like(v), np.zeros_like(v), 1, 2e-3, 1e-4)
        else:
            p1 = stats[k]
        out["new256:" + k] = p1.reshape(-1)[:256]
    w32 = {k: v.astype(np.float32) for k, v in w.items()}
    prob32, cache32, _ = orc.forward(w32, x.astype(np.float32), training=True, drop_seeds=seeds)
    _, dprob32 = orc.loss_and_dprob(y.astype(np.float32), prob32)
    del prob32
    g32, _ = orc.backward(w32, cache32, dprob32)
    del cache32
    for k, v in g.items():
        a, b = g32[k].reshape(-1).astype(np.float64), v.reshape(-1)
        out["e32:" + k] = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        i = sub_index(b.size)
        out["e32sub:" + k] = np.linalg.norm(a[i] - b[i]) / max(np.linalg.norm(b[i]), 1e-30)
        l32, s32 = channel_norms(g32[k])
        out["e32cn_last:" + k] = rel_l2(l32, out["cn_last:" + k])
        out["e32cn_sec:" + k] = rel_l2(s32, out["cn_sec:" + k])
    return out


def train256_fixture():
    """configs[1]: 256x256x3 binary, batch 16 (the geometry scripts/train.py trains at, :84-88)."""
    return train_big_fixture(256, 16, 1, 51, 11)


def train256c21_fixture():
    """configs[4] per GPU: 256x256x3, 21 classes (softmax head), batch 8."""
    return train_big_fixture(256, 8, 21, 61, 12)


def train512_fixture():
    """configs[3] per GPU: 512x512x3 binary, batch 8 (the HBM-bound regime BASELINE.json names)."""
    return train_big_fixture(512, 8, 1, 71, 13)


def train256d_fixture():
    """configs[1] as the reference trains and bench.py times it: 256x256x3 binary, batch 16, with
    U_NET's default dropout_rate=0.2 (model/u_net.py:30, scripts/train.py:223) at the bottleneck and
    dec4 / dec3 / dec2 (:77-78, 97-98); masks from the engine's step-1 seeds (engine_seed 2301)."""
    return train_big_fixture(256, 16, 1, 81, 14, drop=0.2)


def train256b32_fixture():
    """configs[4] with its whole batch of 32 on one GPU (21 classes, 256x256x3, dropout 0.2): the batch
    that routes the 32x32 level through the fused split-precision forward (engine FUSE_MIN_TOTAL_PIXELS;
    the encoder table's batch, model/u_net.py:63-69)."""
    return train_big_fixture(256, 32, 21, 91, 15, drop=0.2)


def write(name, d):
    np.savez_compressed(os.path.join(HERE, name), **{k.replace("/", "|"): v for k, v in d.items()})


BIG = {"fwd256.npz": fwd256_fixture, "fwd512.npz": fwd512_fixture, "fwd21.npz": fwd21_fixture,
       "samples.npz": samples_fixture, "train128.npz": train128_fixture, "train256.npz": train256_fixture,
       "train256c21.npz": train256c21_fixture,
       "train512.npz": train512_fixture, "train256d.npz": train256d_fixture,
       "train256b32.npz": train256b32_fixture}


if __name__ == "__main__" and len(sys.argv) > 1:  # regenerate only the named fixtures
    for nm in sys.argv[1:]:
        write(nm, BIG[nm]())
        print(nm, os.path.getsize(os.path.join(HERE, nm)))
elif __name__ == "__main__":
    for nm, fn in BIG.items():
        write(nm, fn())
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops_fixture())
    np.savez_compressed(os.path.join(HERE, "cfg1_forward.npz"), **cfg1_fixture())
    tf = train_fixture()
    np.savez_compressed(os.path.join(HERE, "train_step.npz"), **{k.replace("/", "|"): v for k, v in tf.items()})
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
