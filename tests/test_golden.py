"""Committed golden vectors (tests/golden/, made by make_golden.py): the oracle must keep
reproducing them (CPU), and the HIP path must match them (GPU)."""
import os

import numpy as np
import pytest

from oracle import keras_ops as K
from oracle.unet_ref import UNetOracle

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
import sys  # noqa: E402
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402


def _load(name):
    with np.load(os.path.join(HERE, name), allow_pickle=False) as z:
        return {k.replace("|", "/"): z[k] for k in z.files}


def test_oracle_reproduces_op_goldens():
    g = _load("ops.npz")
    new = MG.ops_fixture()
    assert set(g) == set(new)
    for k in g:
        assert np.allclose(new[k], g[k], rtol=1e-12, atol=1e-14), k


def test_oracle_reproduces_cfg1_golden():
    g = _load("cfg1_forward.npz")
    new = MG.cfg1_fixture()
    assert np.abs(new["prob"].astype(np.float64) - g["prob"]).max() < 1e-6


def test_oracle_reproduces_train_golden():
    g = _load("train_step.npz")
    new = MG.train_fixture()
    for k, v in g.items():
        assert np.allclose(new[k], v, rtol=1e-9, atol=1e-15), k


SLOW = ("train256.npz", "train256c21.npz", "train512.npz", "train256d.npz",
        "train256b32.npz")  # 4-20 min of float64 oracle each: checked below


@pytest.mark.parametrize("name", sorted(set(MG.BIG) - set(SLOW)))
def test_oracle_reproduces_baseline_size_goldens(name):
    """The BASELINE-geometry fixtures (fwd256/fwd512/fwd21/samples/train128) are reproduced by
    the oracle (float64 rounding only)."""
    g = _load(name)
    new = {k.replace("|", "/"): v for k, v in MG.BIG[name]().items()}
    assert set(g) == set(new)
    for k, v in g.items():
        a, b = np.asarray(new[k], np.float64), np.asarray(v, np.float64)
        assert a.shape == b.shape, k
        assert np.allclose(a, b, rtol=1e-9, atol=1e-12), k


@pytest.mark.parametrize("name", SLOW)
def test_training_geometry_goldens_consistent(name):
    """The 256x256 train-step fixtures (regenerate: python tests/golden/make_golden.py NAME):
    every variable and block present, dice = 1 - loss, the subsample and first values agree
    with the norms, and the stored post-AdamW values are the oracle's AdamW of the stored
    gradients on the documented weights."""
    from oracle import keras_ops as K
    from unet_amd.params import unet_variables
    g = _load(name)
    ncls = int(g["ncls"])
    specs = unet_variables(3, ncls)
    trainable = {s.name for s in specs if s.trainable}
    assert {k[6:] for k in g if k.startswith("gnorm:")} == trainable
    assert {k[7:] for k in g if k.startswith("new256:")} == {s.name for s in specs}
    assert len([k for k in g if k.startswith("bn_mean:")]) == 18
    assert abs(float(g["dice"]) + float(g["loss"]) - 1.0) < 1e-12
    if float(g.get("drop", 0.0)) > 0:  # the dropout masks are the engine's step-1 draws
        seeds = MG.engine_drop_seeds(int(g["engine_seed"]), 1)
        assert {k[10:]: int(v) for k, v in g.items() if k.startswith("drop_seed:")} == seeds
    w = MG.model_weights(ncls, MG.FULL, int(g["w_seed"]))
    for k in trainable:
        sub = g["gsub:" + k].astype(np.float64)
        assert np.linalg.norm(sub) <= float(g["gnorm:" + k]) * (1 + 1e-6) + 1e-30
        n = min(128, g["g128:" + k].size)
        w0 = w[k].reshape(-1)[:n]
        p1, _, _ = K.adamw_update(w0, g["g128:" + k][:n], np.zeros(n), np.zeros(n), 1, 2e-3, 1e-4)
        assert np.allclose(p1, g["new256:" + k][:n], rtol=1e-12, atol=1e-15), k
        assert 0.0 <= float(g["e32sub:" + k]) < 0.1 and 0.0 <= float(g["e32:" + k]) < 0.1, k
        # per-channel norms: one per channel of each axis, and each axis's norms square-sum to
        # the tensor norm
        shape = next(s.shape for s in specs if s.name == k)
        last, sec = g["cn_last:" + k], g["cn_sec:" + k]
        if len(shape) >= 2:
            assert last.shape == (shape[-1],) and sec.shape == (shape[-2],), k
        for v in (last, sec):
            assert abs(np.linalg.norm(v) - float(g["gnorm:" + k])) <= 1e-9 * float(g["gnorm:" + k]) + 1e-30, k
        assert 0.0 <= float(g["e32cn_last:" + k]) < 0.1 and 0.0 <= float(g["e32cn_sec:" + k]) < 0.1, k


def test_gradient_subsample_hits_every_channel():
    """the training-geometry subsample covers every output channel and every
    input channel of each large pointwise / Conv2DTranspose kernel (so every MFMA lane / column of
    a tile is checked), not only the channels that are multiples of the old stride."""
    from unet_amd.params import unet_variables
    for ncls in (1, 21):
        for s in unet_variables(3, ncls, True, MG.FULL):
            n = int(np.prod(s.shape))
            i = MG.sub_index(n)
            assert np.unique(i).size == i.size == min(n, MG.SUB)
            if len(s.shape) >= 2 and s.shape[-1] > 1:
                assert np.unique(i % s.shape[-1]).size == s.shape[-1], s.name
                assert np.unique((i // s.shape[-1]) % s.shape[-2]).size == s.shape[-2], s.name
                # every residue mod 32 of both channel axes
                for ax, c in ((i % s.shape[-1], s.shape[-1]), ((i // s.shape[-1]) % s.shape[-2], s.shape[-2])):
                    if c >= 32:
                        assert np.bincount(ax % 32, minlength=32).min() > 0, s.name


@pytest.mark.gpu
def test_hip_matches_cfg1_golden():
    """configs[0] through the reference builder API: masks within 1e-3 of the golden output."""
    from model.u_net import U_NET
    g = _load("cfg1_forward.npz")
    model = U_NET((128, 128, 3), 1)
    w = MG.model_weights(1, (64, 128, 256, 512), int(g["w_seed"]))
    model.engine.set_weights_dict({k: v.astype(np.float32) for k, v in w.items()})
    x = MG.U(int(g["x_seed"]), (2, 128, 128, 3)).astype(np.float32)
    prob = model.predict(x)
    err = np.abs(prob.astype(np.float64) - g["prob"]).max()
    assert err < 1e-3
    assert err < 2e-5


@pytest.mark.gpu
def test_hip_matches_train_golden():
    import torch
    from unet_amd.model import UNetModel
    from unet_amd.optim import AdamW
    g = _load("train_step.npz")
    m = UNetModel((32, 32, 3), 1, dropout_rate=0.0)
    w = MG.model_weights(1, (64, 128, 256, 512), int(g["w_seed"]))
    m.engine.set_weights_dict({k: v.astype(np.float32) for k, v in w.items()})
    x = MG.U(int(g["x_seed"]), (2, 32, 32, 3)).astype(np.float32)
    y = (MG.U(int(g["y_seed"]), (2, 32, 32, 1)) > 0.6).astype(np.float32)
    m.compile(AdamW(2e-3, 1e-4), "dice_loss")
    res = m.train_step(x, y).cpu().numpy()
    torch.cuda.synchronize()
    assert abs(res[0] - g["loss"]) < 1e-5 and abs(res[1] - g["dice"]) < 1e-5
    for k, v in g.items():
        if k.startswith("gnorm:"):
            name = k[6:]
            hn = float(np.linalg.norm(m.engine.gvars[name].cpu().numpy().astype(np.float64)))
            assert abs(hn - v) <= 1e-3 * v + 1e-12, (name, hn, float(v))
    neww = m.engine.get_weights_dict()
    for k, v in g.items():
        if k.startswith("new:"):
            name = k[4:]
            assert np.abs(neww[name] - v).max() <= 1e-4 * np.abs(v).max(), name
