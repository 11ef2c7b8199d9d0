"""The depthwise data gradient of a BN+ReLU-view block that also accumulates the layer's depthwise
FILTER gradient (unet_dwconv3x3_bwd_data_bnstats_dwf + unet_reduce_slabs, ABI 12, round 6) against
the separate launches and the float64 oracle: dx bitwise equal to the plain data gradient, the BN-
backward statistics bitwise equal to the non-filter launch's, the filter gradient within 1e-5 of
float64 (oracle/keras_ops.py depthwise3x3_bwd), at ragged tiles and every channel-quad tiling.

Reference: model/u_net.py:14-25 (SeparableConv2D depthwise half -> BatchNormalization -> ReLU)."""
import numpy as np
import pytest

from helpers import bn_affine, dev, f32, host, rel_err
from oracle import keras_ops as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ops():
    from unet_amd import ops as O
    return O


@pytest.mark.parametrize("use_bn", [True, False])
@pytest.mark.parametrize("n,h,w,c", [(2, 16, 16, 128), (1, 9, 21, 64), (3, 8, 40, 32), (2, 5, 7, 8), (1, 33, 17, 4),
                                     (2, 32, 32, 256)])
def test_dwconv_bwd_data_bnstats_dwf(ops, use_bn, n, h, w, c):
    rng = np.random.default_rng(n * 1000 + h * 10 + w + c + use_bn)
    z = f32(rng.standard_normal((n, h, w, c)))
    sc, sh = bn_affine(rng, c)
    v = ops.View.bnrelu(dev(z), dev(sc), dev(sh))
    dk = f32(rng.standard_normal((3, 3, c, 1)))
    dy = f32(rng.standard_normal((n, h, w, c)))
    S = ops.dwconv3x3_bwd_data_bnstats_slabs(v, n, h, w)
    assert S > 0
    mean = dev(f32(rng.standard_normal(c) * 0.1))
    rstd = dev(f32(1.0 + rng.random(c)))
    mu, rs = (mean, rstd) if use_bn else (None, None)
    m = n * h * w
    res = {}
    for fused in (True, False):
        part = torch.zeros(ops.bn_stats_partials_numel(S, c), device="cuda")
        dx = torch.full((n, h, w, c), 7.0, device="cuda")
        if fused:
            slabs = torch.full((S * 9 * c,), 3.0, device="cuda")
            ops.dwconv3x3_bwd_data_bnstats_dwf(v, n, h, w, dev(dk), dev(dy), dx, mu, rs, part, slabs)
            ddk = torch.full((3, 3, c, 1), 5.0, device="cuda")
            ops.reduce_slabs(slabs, S, 9 * c, ddk)
        else:
            ops.dwconv3x3_bwd_data_bnstats(v, n, h, w, dev(dk), dev(dy), dx, mu, rs, part)
            ddk = torch.full((3, 3, c, 1), 5.0, device="cuda")
            ops.dwconv3x3_bwd_filter(v, n, h, w, dev(dy), ddk)
        dg, db, coef = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda"), torch.empty(3 * c, device="cuda")
        ops.bn_relu_bwd_stats_finish(part, S, m, c, mu, rs, use_bn, dg if use_bn else None, db, coef)
        res[fused] = (host(dx), host(db), host(dg), host(coef), host(ddk))
    for i in range(4):  # dx and the statistics: the same arithmetic in both launches
        assert np.array_equal(res[True][i], res[False][i]), i
    x = np.maximum(z.astype(np.float64) * sc + sh, 0)
    _, rdk = K.depthwise3x3_bwd(x, dk.astype(np.float64), dy.astype(np.float64))
    assert rel_err(res[True][4], rdk) < 1e-5
    assert rel_err(res[True][4], res[False][4].astype(np.float64)) < 1e-5
