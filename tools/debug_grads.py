"""Localise a gradient mismatch: per-block dA (grad w.r.t. block output) HIP vs oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np, torch
from helpers import norm_err
from oracle.unet_ref import UNetOracle
from unet_amd.model import UNetModel
from test_model_gpu import _weights_with_stats, _data
ncls = int(sys.argv[1]) if len(sys.argv) > 1 else 21
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 32
model = UNetModel((hw, hw, 3), ncls, dropout_rate=0.0, seed=11)
rng = np.random.default_rng(ncls * 13 + 1)
p = _weights_with_stats(model, rng)
x, y = _data(rng, 2, hw, hw, ncls)
xt, yt = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
res = model.engine.forward_train(xt, yt)
model.engine.backward(yt, 0)
torch.cuda.synchronize()
A = model.engine._acts_last
orc = UNetOracle(ncls, 0.0)
prob, cache, _ = orc.forward(p, x.astype(np.float64), training=True)
l, dp = orc.loss_and_dprob(y.astype(np.float64), prob)
trace = {}
g, _ = orc.backward(p, cache, dp, trace)
print("prob err", np.abs(A.prob.cpu().numpy() - prob).max(), "loss", res.cpu().numpy()[0], l)
for b in model.engine.blocks:
    hda = A.blocks[b.name].da.cpu().numpy().astype(np.float64)
    print(f"{b.name:15s} dA err {norm_err(hda, trace[b.name]):.3e}   |dA| {np.linalg.norm(trace[b.name]):.3e}")
for k in ("enc2_block2_bn/gamma", "enc2_block2_sepconv/pointwise_kernel", "enc2_block1_bn/gamma"):
    print(k, norm_err(model.engine.gvars[k].cpu().numpy(), g[k]))
errs = sorted(((norm_err(model.engine.gvars[k].cpu().numpy(), g[k]), k) for k in g))
print("smallest:", errs[:5])
print("largest:", errs[-5:])
