"""Per-op parity of the HIP kernels (through the C-ABI) against the NumPy oracle (float64),
on seeded inputs at small shapes, including tails (pixel counts that are not a multiple of
the 128-row tile, 3-channel inputs, 3-channel outputs) and every activation-view mode."""
import numpy as np
import pytest

from helpers import bn_affine, dev, f32, host, norm_err, rel_err, view_value
from oracle import keras_ops as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ops():
    from unet_amd import ops as O
    return O


def _mk_view(O, mode, t, drop_rate=0.0, drop_seed=0):
    """t: dict of device tensors -> ops.View"""
    if mode == 0:
        v = O.View.plain(t["src0"])
    elif mode == 1:
        v = O.View.bnrelu(t["src0"], t["sc0"], t["sh0"])
    elif mode == 2:
        v = O.View.pool_bnrelu(t["src0"], t["sc0"], t["sh0"])
    else:
        v = O.View.concat(t["src0"], t["src1"], t["sc1"], t["sh1"])
    return v.dropout(drop_rate, drop_seed) if drop_rate > 0 else v


def _view_inputs(rng, mode, n, h, w, c0, c1=0):
    """Returns (numpy dict, device dict) of the view sources for logical dims (n,h,w)."""
    a = {}
    if mode == 2:
        a["src0"] = f32(rng.standard_normal((n, 2 * h, 2 * w, c0)))
    else:
        a["src0"] = f32(rng.standard_normal((n, h, w, c0)))
    if mode in (1, 2):
        a["sc0"], a["sh0"] = bn_affine(rng, c0)
    if mode == 3:
        a["src1"] = f32(rng.standard_normal((n, h, w, c1)))
        a["sc1"], a["sh1"] = bn_affine(rng, c1)
    return a, {k: dev(v) for k, v in a.items()}


VIEW_CASES = [
    # mode, n, h, w, c0, c1, drop
    (0, 2, 9, 7, 3, 0, 0.0),      # image input: 3 channels, scalar path, ragged pixels
    (0, 2, 16, 16, 16, 0, 0.0),
    (1, 2, 12, 10, 32, 0, 0.0),
    (2, 2, 8, 8, 16, 0, 0.0),
    (3, 2, 8, 6, 16, 16, 0.0),
    (3, 2, 8, 8, 8, 8, 0.2),      # decoder concat with dropout
    (1, 1, 4, 4, 64, 0, 0.2),
]


@pytest.mark.parametrize("mode,n,h,w,c0,c1,drop", VIEW_CASES)
def test_view_materialize(ops, mode, n, h, w, c0, c1, drop):
    rng = np.random.default_rng(10 + mode)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    v = _mk_view(ops, mode, t, drop, 1234)
    out = torch.empty((n, h, w, c0 + c1), device="cuda")
    ops.view_materialize(v, n, h, w, out)
    ref = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"),
                     drop, 1234)
    assert rel_err(host(out), ref) < 1e-6


@pytest.mark.parametrize("mode,n,h,w,c0,c1,drop", VIEW_CASES)
def test_dwconv_fwd(ops, mode, n, h, w, c0, c1, drop):
    rng = np.random.default_rng(20 + mode)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk = f32(rng.standard_normal((3, 3, C, 1)))
    v = _mk_view(ops, mode, t, drop, 99)
    y = torch.empty((n, h, w, C), device="cuda")
    ops.dwconv3x3_fwd(v, n, h, w, dev(dk), y)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"), drop, 99)
    assert rel_err(host(y), K.depthwise3x3(xv, dk)) < 2e-6


@pytest.mark.parametrize("mode,n,h,w,c0,c1,drop", VIEW_CASES)
def test_dwconv_bwd(ops, mode, n, h, w, c0, c1, drop):
    rng = np.random.default_rng(30 + mode)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk = f32(rng.standard_normal((3, 3, C, 1)))
    dy = f32(rng.standard_normal((n, h, w, C)))
    v = _mk_view(ops, mode, t, drop, 7)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"), drop, 7)
    dxv, ddk = K.depthwise3x3_bwd(xv, dk, dy)
    if drop > 0:
        dxv = dxv * K.dropout_mult(7, dxv.shape, drop)
    # filter gradient
    g = torch.empty((3, 3, C, 1), device="cuda")
    ops.dwconv3x3_bwd_filter(v, n, h, w, dev(dy), g)
    assert rel_err(host(g), ddk) < 1e-5
    # data gradient, routed per view mode
    if mode in (0, 1):
        dx0 = torch.empty((n, h, w, C), device="cuda")
        ops.dwconv3x3_bwd_data(v, n, h, w, dev(dk), dev(dy), dx0)
        assert rel_err(host(dx0), dxv) < 2e-6
    elif mode == 3:
        dx0 = torch.empty((n, h, w, c0), device="cuda")
        dx1 = torch.empty((n, h, w, c1), device="cuda")
        ops.dwconv3x3_bwd_data(v, n, h, w, dev(dk), dev(dy), dx0, dx1)
        assert rel_err(host(dx0), dxv[..., :c0]) < 2e-6
        assert rel_err(host(dx1), dxv[..., c0:]) < 2e-6
    else:
        init = f32(rng.standard_normal((n, 2 * h, 2 * w, c0)))
        dx0 = dev(init)
        ops.dwconv3x3_bwd_data(v, n, h, w, dev(dk), dev(dy), dx0)
        act = K.relu(a["src0"] * a["sc0"] + a["sh0"])
        ref = init + K.maxpool2_bwd(act, dxv)
        assert rel_err(host(dx0), ref) < 2e-6


@pytest.mark.parametrize("m,cin,cout,off", [(100, 3, 64, 0.0), (256, 64, 64, 0.0), (300, 64, 128, 0.0),
                                            (128, 128, 256, 0.0), (77, 32, 96, 0.0), (512, 256, 512, 0.0),
                                            # > 64 partials: several finalize chunks; |mean| >> std
                                            (24653, 64, 64, 0.0), (24653, 32, 128, 25.0)])
def test_pointwise_and_bn_stats(ops, m, cin, cout, off):
    rng = np.random.default_rng(m + cin)
    y = f32(rng.standard_normal((m, cin)) + off)
    pk = f32(rng.standard_normal((1, 1, cin, cout)) / np.sqrt(cin))
    z = torch.empty((m, cout), device="cuda")
    part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
    ops.pointwise_fwd(dev(y), m, cin, cout, dev(pk), z, part)
    zr = y @ pk[0, 0]
    assert rel_err(host(z), zr) < 5e-6
    gamma, beta = bn_affine(rng, cout)
    mm = f32(rng.standard_normal(cout) * 0.1)
    mv = f32(1 + rng.random(cout))
    tm, tv = dev(mm), dev(mv)
    outs = [torch.empty(cout, device="cuda") for _ in range(4)]
    ops.bn_finalize(part, m, cout, dev(gamma), dev(beta), 1e-3, 0.99, tm, tv, True, *outs)
    zz = zr[:, None, None, :].reshape(m, 1, 1, cout)
    out, mean, var = K.bn_train(zz, gamma, beta)
    mm2, mv2 = K.bn_moving_update(mm, mv, mean, var)
    inv = gamma / np.sqrt(var + 1e-3)
    assert rel_err(host(outs[0]), mean) < 1e-4
    assert rel_err(host(outs[1]), 1 / np.sqrt(var + 1e-3)) < 1e-5
    assert rel_err(host(outs[2]), inv) < 1e-5
    assert rel_err(host(outs[3]), beta - mean * inv) < 1e-4
    assert rel_err(host(tm), mm2) < 1e-5 and rel_err(host(tv), mv2) < 1e-5
    # again: the finalize's arrival counters were left zero, the result is bitwise the same
    outs2 = [torch.empty(cout, device="cuda") for _ in range(4)]
    ops.bn_finalize(part, m, cout, dev(gamma), dev(beta), 1e-3, 0.99, None, None, False, *outs2)
    assert all(torch.equal(a, b) for a, b in zip(outs, outs2))
    assert not torch.any(part[-((cout + 63) // 64):].view(torch.int32))
    # no-partials path (inference GEMM epilogue)
    z2 = torch.empty((m, cout), device="cuda")
    ops.pointwise_fwd(dev(y), m, cin, cout, dev(pk), z2, None)
    assert torch.equal(z, z2)


@pytest.mark.parametrize("rows,cout,off", [((3000, 2000), 64, 0.0), ((24653, 9000), 128, 25.0),
                                           ((128, 129, 1000), 96, 1.0), ((5000,), 256, 0.0)])
def test_bn_sync_moments(ops, rows, cout, off):
    """SyncBN forward (unet_bn_moments + unet_bn_finalize_moments): the replicas' records combined in
    rank order give the statistics of the concatenated batch -- against unet_bn_finalize over all
    rows and the float64 oracle; one replica reproduces unet_bn_finalize.  Backward coefficients
    (unet_bn_bwd_coef) = (mean, S1 / m, rstd S2 / m)."""
    rng = np.random.default_rng(sum(rows) + cout)
    cin = 32
    pk = f32(rng.standard_normal((1, 1, cin, cout)) / np.sqrt(cin))
    ys = [f32(rng.standard_normal((r, cin)) + off) for r in rows]
    gamma, beta = bn_affine(rng, cout)
    mm = f32(rng.standard_normal(cout) * 0.1)
    mv = f32(1 + rng.random(cout))
    R = 1 + 2 * cout
    recs = torch.empty(len(rows) * R, dtype=torch.float64, device="cuda")
    for i, (r, y) in enumerate(zip(rows, ys)):
        z = torch.empty((r, cout), device="cuda")
        part = torch.zeros(ops.bn_partials_numel(r, cout), device="cuda")
        ops.pointwise_fwd(dev(y), r, cin, cout, dev(pk), z, part)
        ops.bn_moments(part, r, cout, recs[i * R:(i + 1) * R])
    tm, tv = dev(mm), dev(mv)
    outs = [torch.empty(cout, device="cuda") for _ in range(4)]
    ops.bn_finalize_moments(recs, len(rows), cout, dev(gamma), dev(beta), 1e-3, 0.99, tm, tv, True, *outs)
    # reference: one replica holding every row
    M = sum(rows)
    yall = np.concatenate(ys)
    zall = torch.empty((M, cout), device="cuda")
    pall = torch.zeros(ops.bn_partials_numel(M, cout), device="cuda")
    ops.pointwise_fwd(dev(yall), M, cin, cout, dev(pk), zall, pall)
    tm2, tv2 = dev(mm), dev(mv)
    ref = [torch.empty(cout, device="cuda") for _ in range(4)]
    ops.bn_finalize(pall, M, cout, dev(gamma), dev(beta), 1e-3, 0.99, tm2, tv2, True, *ref)
    for a, b in zip(outs + [tm, tv], ref + [tm2, tv2]):
        assert rel_err(host(a), host(b)) < 2e-6
    zr = (yall @ pk[0, 0]).reshape(M, 1, 1, cout)
    _, mean, var = K.bn_train(zr, gamma, beta)
    assert rel_err(host(outs[0]), mean) < 1e-4
    assert rel_err(host(outs[1]), 1 / np.sqrt(var + 1e-3)) < 1e-5
    # backward coefficients from (all-reduced) sums
    sums = dev(f32(rng.standard_normal(2 * cout)))
    coef = torch.empty(3 * cout, device="cuda")
    ops.bn_bwd_coef(sums, M, cout, True, outs[0], outs[1], coef)
    sh = host(sums)
    want = np.concatenate([host(outs[0]), sh[:cout] / M, host(outs[1]) * (sh[cout:] / M)])
    assert rel_err(host(coef), want) < 1e-6


@pytest.mark.parametrize("m,cin,cout", [(100, 3, 64), (256, 64, 64), (300, 128, 64), (200, 256, 512),
                                        (64, 1024, 1024)])
def test_pointwise_bwd(ops, m, cin, cout):
    rng = np.random.default_rng(m * 3 + cout)
    y = f32(rng.standard_normal((m, cin)))
    pk = f32(rng.standard_normal((1, 1, cin, cout)) / np.sqrt(cin))
    dz = f32(rng.standard_normal((m, cout)))
    dy = torch.empty((m, cin), device="cuda")
    ops.pointwise_bwd_data(dev(dz), m, cin, cout, dev(pk), dy)
    dpk = torch.empty((1, 1, cin, cout), device="cuda")
    ops.pointwise_bwd_filter(dev(y), dev(dz), m, cin, cout, dpk)
    ry, rpk = K.pointwise_bwd(y.reshape(m, 1, 1, cin), pk, dz.reshape(m, 1, 1, cout))
    assert rel_err(host(dy), ry.reshape(m, cin)) < 5e-6
    assert rel_err(host(dpk), rpk) < 5e-6


@pytest.mark.parametrize("use_bn,drop", [(True, 0.0), (True, 0.2), (False, 0.0)])
@pytest.mark.parametrize("m,c", [(300, 16), (1000, 64), (96, 3)])
def test_bn_relu_bwd(ops, use_bn, drop, m, c):
    rng = np.random.default_rng(m + c)
    z = f32(rng.standard_normal((m, 1, 1, c)) * 2 + 0.3)
    da = f32(rng.standard_normal((m, 1, 1, c)))
    gamma, beta = bn_affine(rng, c)
    if use_bn:
        _, mean, var = K.bn_train(z, gamma, beta)
        rstd = 1 / np.sqrt(var + 1e-3)
        scale = f32(gamma * rstd)
        shift = f32(beta - mean * gamma * rstd)
    else:
        mean = var = rstd = np.zeros(c)
        scale, shift = np.ones(c), beta
    dmult = K.dropout_mult(55, da.shape, drop) if drop > 0 else None
    dg = torch.zeros(c, device="cuda")
    db = torch.zeros(c, device="cuda")
    dz = torch.empty((m, c), device="cuda")
    ops.bn_relu_bwd(dev(da), dev(z), m, c, dev(f32(mean)), dev(f32(rstd)), dev(scale), dev(shift), use_bn, drop, 55,
                    dg if use_bn else None, db, dz)
    if use_bn:
        rz, rg, rb = K.bn_relu_bwd(da, z, gamma, beta, f32(mean), f32(var), drop=dmult)
        assert rel_err(host(dg), rg) < 1e-4
    else:
        g = da if dmult is None else da * dmult
        rz = np.where(z + beta > 0, g, 0)
        rb = rz.reshape(-1, c).sum(0)
    assert rel_err(host(db), rb) < 1e-5
    assert rel_err(host(dz), rz.reshape(m, c)) < 1e-4


@pytest.mark.parametrize("use_bn", [True, False])
@pytest.mark.parametrize("m,cout", [(300, 64), (37, 32), (1000, 32), (40000, 64), (300000, 64)])  # ragged; 2048 slabs
def test_pointwise_bwd_data_bnrelu_wgrad(ops, use_bn, m, cout):
    """Image block (cin 4): data gradient plus the pointwise weight gradient from the dz formed on the
    fly (dz never stored): dy against the GEMM launch, dW against the float64 oracle
    sum_m y[m, ci] dz[m, co] and against the stored-dz weight-gradient launch."""
    rng = np.random.default_rng(m + 3 * cout + use_bn)
    cin, c = 4, cout
    z = f32(rng.standard_normal((m, c)) * 2 + 0.3)
    da = f32(rng.standard_normal((m, c)))
    y = f32(rng.standard_normal((m, cin)))
    y[:, 3] = 0.0  # the padded image channel
    pk = f32(rng.standard_normal((1, 1, cin, cout)) / np.sqrt(cout))
    gamma, beta = bn_affine(rng, c)
    if use_bn:
        mean, var = z.mean(0), z.var(0)
        rstd = 1 / np.sqrt(var + 1e-3)
        scale, shift = f32(gamma * rstd), f32(beta - mean * gamma * rstd)
    else:
        mean = rstd = np.zeros(c)
        scale, shift = f32(np.ones(c)), beta
    dg, db, coef = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda"), torch.empty(3 * c, device="cuda")
    ts, th = dev(scale), dev(shift)
    ops.bn_relu_bwd_stats(dev(da), dev(z), m, c, dev(f32(mean)), dev(f32(rstd)), ts, th, use_bn, 0.0, 0,
                          dg if use_bn else None, db, coef)
    dy_f, dy_p = torch.empty((m, cin), device="cuda"), torch.empty((m, cin), device="cuda")
    dpk_f, dpk_p = torch.full((1, 1, cin, cout), 7.0, device="cuda"), torch.empty((1, 1, cin, cout), device="cuda")
    dz = torch.empty((m, c), device="cuda")
    ops.pointwise_bwd_data_bnrelu_wgrad(dev(da), dev(z), m, cin, cout, dev(pk), ts, th, coef, dev(y), dy_f, dpk_f)
    assert ops.L.query("unet_pointwise_bwd_data_bnrelu_wgrad_workspace", m, cin, 48) == 0
    ops.pointwise_bwd_data_bnrelu(dev(da), dev(z), m, cin, cout, dev(pk), ts, th, coef, 0.0, 0, dy_p, dz)
    assert rel_err(host(dy_f), host(dy_p)) < 1e-5  # (different summation order from the MFMA GEMM)
    ops.pointwise_bwd_filter(dev(y), dz, m, cin, cout, dpk_p)
    assert rel_err(host(dpk_f), host(dpk_p)) < 1e-5
    ref = y.astype(np.float64).T @ host(dz).astype(np.float64)
    assert rel_err(host(dpk_f).reshape(cin, cout), ref) < 1e-5
    assert not torch.any(dpk_f[0, 0, 3])  # zero input channel -> zero gradient row


@pytest.mark.parametrize("cout", [32, 64])
@pytest.mark.parametrize("n,h,w,wcin", [(2, 17, 19, 3), (1, 64, 64, 3), (3, 8, 5, 4), (1, 3, 130, 3)])
def test_image_block_bwd_wgrad(ops, n, h, w, wcin, cout):
    """Both image-block weight gradients in one pass (dy formed and contracted with x's 3x3
    neighbourhood, never stored), in the Keras wcin-channel shapes: against the two-launch path
    (data + pointwise gradient, then the depthwise filter gradient over the stored dy) and the
    float64 restatement of dK[i, j, c] = sum dy[p, c] x[p + (i - 1, j - 1), c] (zero padding)."""
    rng = np.random.default_rng(n * 1000 + h * 10 + w + cout + wcin)
    m, cin, c = n * h * w, 4, cout
    x = f32(rng.standard_normal((n, h, w, cin)))
    x[..., wcin:] = 0.0
    z = f32(rng.standard_normal((m, c)) * 2 + 0.3)
    da = f32(rng.standard_normal((m, c)))
    y = f32(rng.standard_normal((m, cin)))
    y[:, wcin:] = 0.0
    pk = f32(rng.standard_normal((1, 1, cin, cout)) / np.sqrt(cout))
    pk[:, :, wcin:] = 0.0
    gamma, beta = bn_affine(rng, c)
    mean, var = z.mean(0), z.var(0)
    rstd = 1 / np.sqrt(var + 1e-3)
    ts, th = dev(f32(gamma * rstd)), dev(f32(beta - mean * gamma * rstd))
    dg, db, coef = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda"), torch.empty(3 * c, device="cuda")
    ops.bn_relu_bwd_stats(dev(da), dev(z), m, c, dev(f32(mean)), dev(f32(rstd)), ts, th, True, 0.0, 0, dg, db, coef)
    ddk = torch.full((3, 3, wcin, 1), 7.0, device="cuda")
    dpk = torch.full((1, 1, wcin, cout), 7.0, device="cuda")
    tx = dev(x)
    ops.image_block_bwd_wgrad(tx, n, h, w, wcin, cout, dev(pk), ts, th, coef, dev(da), dev(z), dev(y), ddk, dpk)
    assert ops.L.query("unet_image_block_bwd_wgrad_workspace", n, h, w, 48) == 0
    dy = torch.empty((m, cin), device="cuda")
    dpk_p = torch.empty((1, 1, cin, cout), device="cuda")
    ops.pointwise_bwd_data_bnrelu_wgrad(dev(da), dev(z), m, cin, cout, dev(pk), ts, th, coef, dev(y), dy, dpk_p)
    assert rel_err(host(dpk), host(dpk_p)[:, :, :wcin]) < 1e-5
    ddk_p = torch.empty((3, 3, cin, 1), device="cuda")
    ops.dwconv3x3_bwd_filter(ops.View.plain(tx), n, h, w, dy, ddk_p)
    assert rel_err(host(ddk), host(ddk_p)[:, :, :wcin]) < 1e-5
    g = host(dy).astype(np.float64).reshape(n, h, w, cin)
    xp = np.pad(x.astype(np.float64), ((0, 0), (1, 1), (1, 1), (0, 0)))
    ref = np.stack([np.stack([(g * xp[:, i:i + h, j:j + w]).sum((0, 1, 2)) for j in range(3)]) for i in range(3)])
    assert rel_err(host(ddk)[..., 0], ref[..., :wcin]) < 1e-5


@pytest.mark.parametrize("use_bn,drop", [(True, 0.0), (True, 0.2), (False, 0.0)])
@pytest.mark.parametrize("m,cin,cout", [(300, 16, 32), (1000, 64, 128), (257, 128, 64), (128, 4, 8),
                                       (520, 1024, 64)])  # cin >= 1024: dz pass + plain GEMM
def test_pointwise_bwd_data_bnrelu(ops, use_bn, drop, m, cin, cout):
    """BN + ReLU (+ dropout) backward folded into the pointwise data-gradient GEMM's operand load,
    against the oracle's bn_relu_bwd followed by the pointwise backward."""
    rng = np.random.default_rng(m + cin + 7 * cout)
    c = cout
    z = f32(rng.standard_normal((m, 1, 1, c)) * 2 + 0.3)
    da = f32(rng.standard_normal((m, 1, 1, c)))
    pk = f32(rng.standard_normal((1, 1, cin, cout)) / np.sqrt(cout))
    gamma, beta = bn_affine(rng, c)
    if use_bn:
        _, mean, var = K.bn_train(z, gamma, beta)
        rstd = 1 / np.sqrt(var + 1e-3)
        scale = f32(gamma * rstd)
        shift = f32(beta - mean * gamma * rstd)
    else:
        mean = var = rstd = np.zeros(c)
        scale, shift = np.ones(c), beta
    dmult = K.dropout_mult(55, da.shape, drop) if drop > 0 else None
    dg = torch.zeros(c, device="cuda")
    db = torch.zeros(c, device="cuda")
    coef = torch.empty(3 * c, device="cuda")
    ts, th = dev(scale), dev(shift)
    ops.bn_relu_bwd_stats(dev(da), dev(z), m, c, dev(f32(mean)), dev(f32(rstd)), ts, th, use_bn, drop, 55,
                          dg if use_bn else None, db, coef)
    dy = torch.empty((m, cin), device="cuda")
    dz = torch.full((m, c), 7.0, device="cuda")
    ops.pointwise_bwd_data_bnrelu(dev(da), dev(z), m, cin, cout, dev(pk), ts, th, coef, drop, 55, dy, dz)
    if use_bn:
        rz, rg, rb = K.bn_relu_bwd(da, z, gamma, beta, f32(mean), f32(var), drop=dmult)
        assert rel_err(host(dg), rg) < 1e-4
    else:
        g = da if dmult is None else da * dmult
        rz = np.where(z + beta > 0, g, 0)
        rb = rz.reshape(-1, c).sum(0)
    assert rel_err(host(db), rb) < 1e-5
    assert rel_err(host(dz), rz.reshape(m, c)) < 1e-4
    ry = rz.reshape(m, c) @ pk[0, 0].T
    assert rel_err(host(dy), ry) < 1e-4



@pytest.mark.parametrize("mode,drop", [(1, 0.0), (1, 0.2), (0, 0.0)])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 4, 4, 64, 32), (2, 3, 5, 32, 16), (1, 8, 8, 128, 64)])
def test_conv_transpose(ops, mode, drop, n, h, w, cin, cout):
    rng = np.random.default_rng(n * h * w + cin)
    a, t = _view_inputs(rng, mode, n, h, w, cin)
    v = _mk_view(ops, mode, t, drop, 4242)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), drop_rate=drop, drop_seed=4242)
    k = f32(rng.standard_normal((2, 2, cout, cin)) / np.sqrt(cin))
    b = f32(rng.standard_normal(cout))
    out = torch.empty((n, 2 * h, 2 * w, cout), device="cuda")
    ops.conv_transpose2x2_fwd(v, n, h, w, cout, dev(k), dev(b), out)
    assert rel_err(host(out), K.conv_transpose2x2(xv, k, b)) < 5e-6
    dout = f32(rng.standard_normal((n, 2 * h, 2 * w, cout)))
    dx = torch.empty((n, h, w, cin), device="cuda")
    dk = torch.empty((2, 2, cout, cin), device="cuda")
    db = torch.empty(cout, device="cuda")
    ops.conv_transpose2x2_bwd(v, n, h, w, cout, dev(k), dev(dout), dx, dk, db)
    rdx, rdk, rdb = K.conv_transpose2x2_bwd(xv, k, dout)
    assert rel_err(host(dx), rdx) < 5e-6
    assert rel_err(host(dk), rdk) < 5e-6
    assert rel_err(host(db), rdb) < 5e-6


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("cin", [32, 64, 128, 256, 48])  # 48: the LDS-tile kernel
@pytest.mark.parametrize("n,h,w", [(2, 12, 10), (1, 3, 5), (3, 64, 40)])  # ragged pixel counts; > 1 grid pass
def test_head_fwd_binary(ops, mode, cin, n, h, w):
    """Binary sigmoid head (u_net.py:105-112) against the float64 oracle."""
    rng = np.random.default_rng(cin + 3 * mode + n * h * w)
    a, t = _view_inputs(rng, mode, n, h, w, cin)
    v = _mk_view(ops, mode, t)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"))
    k = f32(rng.standard_normal((1, 1, cin, 1)) * 0.2)
    b = f32(rng.standard_normal(1) * 0.1)
    prob = torch.full((n, h, w, 1), -1.0, device="cuda")
    ops.head_fwd(v, n, h, w, 1, dev(k), dev(b), prob)
    assert rel_err(host(prob), K.head(xv, k, b, 1)) < 2e-6


@pytest.mark.parametrize("ncls", [1, 21])
@pytest.mark.parametrize("loss_kind", [0, 1])
def test_head_dice(ops, ncls, loss_kind):
    rng = np.random.default_rng(ncls + 7 * loss_kind)
    n, h, w, cin = 2, 12, 10, 64
    a, t = _view_inputs(rng, 1, n, h, w, cin)
    v = _mk_view(ops, 1, t)
    xv = view_value(1, a["src0"], a["sc0"], a["sh0"])
    k = f32(rng.standard_normal((1, 1, cin, ncls)) * 0.2)
    b = f32(rng.standard_normal(ncls) * 0.1)
    prob = torch.empty((n, h, w, ncls), device="cuda")
    ops.head_fwd(v, n, h, w, ncls, dev(k), dev(b), prob)
    rp = K.head(xv, k, b, ncls)
    assert rel_err(host(prob), rp) < 2e-6
    if ncls == 1:
        yt = (rng.random((n, h, w, 1)) > 0.5).astype(np.float64)
    else:
        cls = rng.integers(0, ncls, (n, h, w))
        yt = np.eye(ncls)[cls]
    sums = torch.empty(n * ncls * 3, device="cuda")
    res = torch.empty(3, device="cuda")
    ops.dice_fwd(dev(yt), prob, n, h * w, ncls, 1e-7, sums, res)
    pp = host(prob)
    r = host(res)
    assert abs(r[0] - K.dice_loss(yt, pp)) < 1e-6
    assert abs(r[1] - K.dice_coef(yt, pp)) < 1e-6
    assert abs(r[2] - K.iou_coef(yt, pp)) < 1e-6
    dx = torch.empty((n, h, w, cin), device="cuda")
    dk = torch.empty((1, 1, cin, ncls), device="cuda")
    db = torch.empty(ncls, device="cuda")
    ops.head_bwd(v, n, h, w, ncls, dev(k), prob, dev(yt), sums, 1e-7, loss_kind, dx, dk, db)
    dprob = K.dice_loss_grad(yt, pp) if loss_kind == 0 else K.iou_loss_grad(yt, pp)
    rdx, rdk, rdb = K.head_bwd(xv, k, pp, dprob, ncls)
    assert rel_err(host(dx), rdx) < 1e-4
    assert rel_err(host(dk), rdk) < 1e-4
    assert rel_err(host(db), rdb) < 1e-4
    # loss_scale (data-parallel shard weight) scales every gradient linearly
    ops.head_bwd(v, n, h, w, ncls, dev(k), prob, dev(yt), sums, 1e-7, loss_kind, dx, dk, db, loss_scale=0.75)
    assert rel_err(host(dx), 0.75 * rdx) < 1e-4
    assert rel_err(host(dk), 0.75 * rdk) < 1e-4
    assert rel_err(host(db), 0.75 * rdb) < 1e-4
    with pytest.raises(Exception):
        ops.head_bwd(v, n, h, w, ncls, dev(k), prob, dev(yt), sums, 1e-7, loss_kind, dx, dk, db, loss_scale=0.0)


@pytest.mark.parametrize("ncls", [2, 3, 8, 21, 32])
@pytest.mark.parametrize("cin,mode,nhw,unaligned", [(64, 1, (3, 64, 40), False), (16, 0, (2, 13, 11), False),
                                                    (48, 1, (1, 17, 19), False), (128, 1, (1, 9, 7), False),
                                                    (4, 1, (1, 300, 1), False), (64, 1, (2, 17, 19), False),
                                                    (64, 1, (2, 17, 19), True)])
def test_head_multiclass_shapes(ops, ncls, cin, mode, nhw, unaligned):
    """Softmax head forward + dice-loss backward (u_net.py:105-112, losses) over class counts that
    round up to every register width (4..32), ragged and multi-tile pixel counts, tiles that span
    two images (323 pixels an image), the register kernels (Cin <= 64, Cin/4 dividing 256) and the
    general ones (Cin 48 backward, Cin 128); unaligned: prob and y_true start 4 bytes past a
    16-byte boundary (the scalar staging / store paths)."""
    n, h, w = nhw
    rng = np.random.default_rng(ncls * 131 + cin)
    a, t = _view_inputs(rng, mode, n, h, w, cin)
    v = _mk_view(ops, mode, t)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"))
    k = f32(rng.standard_normal((1, 1, cin, ncls)) * 0.2)
    b = f32(rng.standard_normal(ncls) * 0.1)

    def buf(arr=None):
        size = n * h * w * ncls
        base = torch.full((size + 1,), -1.0, device="cuda")
        out = base[1:] if unaligned else base[:size]
        if arr is not None:
            out.copy_(torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)))
        return out.view(n, h, w, ncls)
    prob = buf()
    ops.head_fwd(v, n, h, w, ncls, dev(k), dev(b), prob)
    pp = host(prob)
    assert rel_err(pp, K.head(xv, k, b, ncls)) < 2e-6
    yt = np.eye(ncls)[rng.integers(0, ncls, (n, h, w))]
    ytd = buf(yt)
    sums = torch.empty(n * ncls * 3, device="cuda")
    res = torch.empty(3, device="cuda")
    ops.dice_fwd(ytd, prob, n, h * w, ncls, 1e-7, sums, res)
    assert abs(host(res)[0] - K.dice_loss(yt, pp)) < 1e-6
    dx = torch.full((n, h, w, cin), 7.0, device="cuda")
    dk = torch.empty((1, 1, cin, ncls), device="cuda")
    db = torch.empty(ncls, device="cuda")
    ops.head_bwd(v, n, h, w, ncls, dev(k), prob, ytd, sums, 1e-7, 0, dx, dk, db)
    rdx, rdk, rdb = K.head_bwd(xv, k, pp, K.dice_loss_grad(yt, pp), ncls)
    assert rel_err(host(dx), rdx) < 1e-4
    assert rel_err(host(dk), rdk) < 1e-4
    assert rel_err(host(db), rdb) < 1e-4


@pytest.mark.parametrize("ncls,thr", [(2, None), (2, 0.5), (5, None), (3, 0.3)])
def test_meaniou(ops, ncls, thr):
    rng = np.random.default_rng(ncls)
    count = 100003
    yt = rng.integers(0, ncls if thr is None else 2, count).astype(np.float64)
    if thr is None:
        yp = rng.random(count) * ncls
        yp[::7] = np.floor(yp[::7])
        yp[::11] = 1.0
    else:
        yp = rng.random(count)
    conf = torch.zeros(ncls * ncls, dtype=torch.int64, device="cuda")
    ops.meaniou_update(dev(yt), dev(yp), ncls, thr, conf)
    ops.meaniou_update(dev(yt), dev(yp), ncls, thr, conf)  # accumulates
    ref = 2 * K.meaniou_confusion(f32(yt), f32(yp), ncls, thr)
    assert np.array_equal(conf.cpu().numpy().reshape(ncls, ncls), ref)
    # buffers not 16-byte aligned take the scalar kernel
    conf.zero_()
    ops.meaniou_update(dev(yt)[1:], dev(yp)[1:], ncls, thr, conf)
    ref = K.meaniou_confusion(f32(yt)[1:], f32(yp)[1:], ncls, thr)
    assert np.array_equal(conf.cpu().numpy().reshape(ncls, ncls), ref)


def test_adamw(ops):
    rng = np.random.default_rng(5)
    n = 10007
    p, g = f32(rng.standard_normal(n)), f32(rng.standard_normal(n) * 0.1)
    m, v = f32(rng.standard_normal(n) * 0.01), f32(rng.random(n) * 0.01)
    tp, tg, tm, tv = dev(p), dev(g), dev(m), dev(v)
    step, lr, wd = 3, 2e-3, 1e-4
    alpha = lr * np.sqrt(1 - 0.999 ** step) / (1 - 0.9 ** step)
    ops.adamw_step(tp, tg, tm, tv, lr, wd, 0.9, 0.999, 1e-7, alpha, 0.5)
    rp, rm, rv = K.adamw_update(p, g * 0.5, m, v, step, lr, wd)
    assert rel_err(host(tp), rp) < 1e-6
    assert rel_err(host(tm), rm) < 1e-6
    assert rel_err(host(tv), rv) < 1e-6


def test_errors_are_loud(ops):
    from unet_amd._lib import UnetHipError
    x = torch.zeros((1, 4, 4, 8), device="cuda")
    with pytest.raises(UnetHipError):  # workspace / shape validation in the C-ABI
        ops.dwconv3x3_fwd(ops.View(1, x, 8), 1, 4, 4, torch.zeros(72, device="cuda"), torch.empty_like(x))
    with pytest.raises(ValueError):
        ops.dwconv3x3_fwd(ops.View.plain(x.cpu()), 1, 4, 4, torch.zeros(72), torch.empty_like(x))


SEP_CASES = [
    # mode, n, h, w, c0, c1, cout, drop
    (0, 2, 16, 32, 16, 0, 64, 0.0),
    (1, 2, 8, 16, 64, 0, 128, 0.0),
    (1, 1, 16, 16, 128, 0, 96, 0.2),
    (2, 2, 8, 16, 32, 0, 64, 0.0),
    (3, 2, 8, 32, 32, 32, 64, 0.0),
    (3, 1, 16, 16, 16, 16, 256, 0.2),
    (1, 1, 8, 16, 8, 0, 8, 0.0),     # K tail (8 channels < 16-channel stage)
    # register-A kernel shapes (>= 64 channels): N tail (192 = 128 + 64), channel-stage tails, concat
    (1, 2, 8, 32, 96, 0, 192, 0.0),
    (3, 1, 16, 16, 64, 68, 64, 0.2),
    (0, 1, 8, 16, 68, 0, 100, 0.0),
    (1, 1, 16, 32, 256, 0, 256, 0.0),
    # max-pool views on the register-A kernel; a grid with several tiles per persistent block
    (2, 2, 8, 16, 64, 0, 128, 0.2),
    (2, 1, 16, 32, 128, 0, 64, 0.0),
    (1, 4, 128, 128, 64, 0, 192, 0.0),
]


@pytest.fixture(params=["auto", "tile"])
def sep_schedule(request, ops):
    old = ops.sepconv_set_schedule(ops.SEPCONV_AUTO if request.param == "auto" else ops.SEPCONV_TILE)
    yield request.param
    ops.sepconv_set_schedule(old)


@pytest.mark.parametrize("mode,n,h,w,c0,c1,cout,drop", SEP_CASES)
@pytest.mark.parametrize("train", [True, False])
def test_fused_sepconv(ops, sep_schedule, mode, n, h, w, c0, c1, cout, drop, train):
    """Both kernel schedules (auto: register-A where it exists; tile: the LDS-A-tile kernel)."""
    rng = np.random.default_rng(100 + mode + cout)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk = f32(rng.standard_normal((3, 3, C, 1)))
    pk = f32(rng.standard_normal((1, 1, C, cout)) / np.sqrt(C))
    v = _mk_view(ops, mode, t, drop, 77)
    assert ops.sepconv_supported(v, n, h, w, cout)
    m = n * h * w
    y = torch.full((n, h, w, C), -7.0, device="cuda")
    z = torch.empty((n, h, w, cout), device="cuda")
    part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
    ops.sepconv_fwd(v, n, h, w, dev(dk), cout, dev(pk), y if train else None, z, part if train else None)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"), drop, 77)
    yr = K.depthwise3x3(xv, dk)
    zr = K.pointwise(yr, pk)
    assert rel_err(host(z), zr) < 5e-6
    if train:
        assert rel_err(host(y), yr) < 2e-6
        outs = [torch.empty(cout, device="cuda") for _ in range(4)]
        gamma, beta = bn_affine(rng, cout)
        ops.bn_finalize(part, m, cout, dev(gamma), dev(beta), 1e-3, 0.99, None, None, False, *outs)
        _, mean, var = K.bn_train(zr, gamma, beta)
        assert rel_err(host(outs[0]), mean) < 1e-4
        assert rel_err(host(outs[1]), 1 / np.sqrt(var + 1e-3)) < 1e-5
    else:
        assert float(y.min()) == -7.0 and float(y.max()) == -7.0  # inference leaves y untouched


@pytest.mark.parametrize("mode,n,h,w,c0,c1,cout,drop", [c for c in SEP_CASES if c[4] + c[5] >= 64])
def test_sepconv_schedules_bitwise_equal(ops, mode, n, h, w, c0, c1, cout, drop):
    """The register-A and LDS-A-tile kernels form every output as the same k-ordered fmaf chain:
    z and y are bitwise equal; the per-tile BN partials (mean, M2) sum the tile's rows in a
    different order (4 waves of 32 rows vs 2 of 64), so they agree to fp32 rounding."""
    rng = np.random.default_rng(7 + cout)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk, pk = dev(rng.standard_normal((3, 3, C, 1))), dev(rng.standard_normal((1, 1, C, cout)) / np.sqrt(C))
    v = _mk_view(ops, mode, t, drop, 5)
    m = n * h * w
    outs = []
    for sch in (ops.SEPCONV_RK, ops.SEPCONV_TILE):
        old = ops.sepconv_set_schedule(sch)
        try:
            y = torch.empty((n, h, w, C), device="cuda")
            z = torch.empty((n, h, w, cout), device="cuda")
            part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
            ops.sepconv_fwd(v, n, h, w, dk, cout, pk, y, z, part)
            torch.cuda.synchronize()
            outs.append((y.cpu(), z.cpu(), part.cpu()))
        finally:
            ops.sepconv_set_schedule(old)
    (y1, z1, p1), (y2, z2, p2) = outs
    assert torch.equal(z1, z2) and torch.equal(y1, y2)
    nb = (m + 127) // 128 * cout * 2
    assert rel_err(p1[:nb].double().numpy(), p2[:nb].double().numpy()) < 1e-6


SW_CASES = [
    # mode, n, h, w, c0, c1, cout, drop
    (1, 2, 8, 16, 64, 0, 64, 0.0),
    (1, 1, 16, 32, 64, 0, 64, 0.2),      # dropout on the view
    (0, 2, 8, 32, 64, 0, 64, 0.0),
    (3, 1, 16, 16, 32, 32, 64, 0.2),     # concat view (decoder), dropout
    (3, 2, 8, 16, 36, 28, 64, 0.0),      # concat with a quad boundary inside the first source
    (3, 1, 16, 32, 64, 64, 64, 0.0),     # two ci groups (dec1_block1: 128 -> 64)
    (3, 1, 8, 16, 128, 128, 64, 0.2),    # four ci groups
    (1, 3, 64, 96, 64, 0, 64, 0.0),      # several tiles per block, ragged tiles per block
    (1, 2, 16, 32, 128, 0, 128, 0.0),    # 128 outputs (the 128 x 128 level: enc2_block2 / dec2_block2)
    (3, 1, 16, 32, 128, 128, 128, 0.2),  # 128 outputs, concat + dropout (dec2_block1: 256 -> 128)
]


@pytest.mark.parametrize("mode,n,h,w,c0,c1,cout,drop", SW_CASES)
def test_sepconv_bwd_filter(ops, mode, n, h, w, c0, c1, cout, drop):
    """Depthwise + pointwise kernel gradients in one pass with y recomputed from the view, against
    the float64 oracle (y = depthwise(view); d_pw = y^T dz; d_dw from depthwise3x3_bwd), and
    against the separate route over the y the fused forward stores."""
    rng = np.random.default_rng(500 + mode + n)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk = f32(rng.standard_normal((3, 3, C, 1)))
    dy = f32(rng.standard_normal((n, h, w, C)))
    dz = f32(rng.standard_normal((n, h, w, cout)))
    v = _mk_view(ops, mode, t, drop, 41)
    assert ops.sepconv_bwd_filter_supported(v, n, h, w, cout)
    ddk = torch.empty((3, 3, C, 1), device="cuda")
    dpk = torch.empty((1, 1, C, cout), device="cuda")
    ops.sepconv_bwd_filter(v, n, h, w, dev(dk), dev(dy), dev(dz), cout, ddk, dpk)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"),
                    drop, 41).astype(np.float64)
    yr = K.depthwise3x3(xv, dk.astype(np.float64))
    _, rpk = K.pointwise_bwd(yr, np.zeros((1, 1, C, cout)), dz.astype(np.float64))
    _, rdk = K.depthwise3x3_bwd(xv, dk.astype(np.float64), dy.astype(np.float64))
    assert rel_err(host(dpk), rpk) < 1e-5
    assert rel_err(host(ddk), rdk) < 1e-5
    y = torch.empty((n, h, w, C), device="cuda")
    ops.sepconv_fwd(v, n, h, w, dev(dk), cout, dev(f32(rng.standard_normal((1, 1, C, cout)))), y,
                    torch.empty((n, h, w, cout), device="cuda"))
    g_pk = torch.empty((1, 1, C, cout), device="cuda")
    g_dk = torch.empty((3, 3, C, 1), device="cuda")
    ops.pointwise_bwd_filter(y, dev(dz), n * h * w, C, cout, g_pk)
    ops.dwconv3x3_bwd_filter(v, n, h, w, dev(dy), g_dk)
    assert rel_err(host(dpk), host(g_pk)) < 2e-6
    assert rel_err(host(ddk), host(g_dk)) < 2e-6


def test_sepconv_bwd_filter_unsupported(ops):
    sc = torch.ones(64, device="cuda")
    x64 = torch.zeros((1, 8, 16, 64), device="cuda")
    assert not ops.sepconv_bwd_filter_supported(ops.View.plain(torch.zeros((1, 8, 16, 96), device="cuda")),
                                                1, 8, 16, 64)  # 96 input channels: not a multiple of 64
    assert not ops.sepconv_bwd_filter_supported(ops.View.plain(x64), 1, 8, 16, 256)  # 256 outputs
    assert not ops.sepconv_bwd_filter_supported(ops.View.pool_bnrelu(torch.zeros((1, 16, 32, 64), device="cuda"),
                                                                     sc, sc), 1, 8, 16, 64)
    with pytest.raises(Exception):
        ops.sepconv_bwd_filter(ops.View.plain(x64), 1, 8, 16, torch.zeros(9 * 64, device="cuda"),
                               torch.zeros(8 * 16 * 64, device="cuda"), torch.zeros(8 * 16 * 256, device="cuda"), 256,
                               torch.empty(9 * 64, device="cuda"), torch.empty(64 * 256, device="cuda"))


def test_sepconv_schedule_rk_refuses_narrow(ops):
    """The register-A kernel needs >= 64 input and output channels; forcing it elsewhere errors."""
    x = torch.zeros((1, 8, 16, 4), device="cuda")
    old = ops.sepconv_set_schedule(ops.SEPCONV_RK)
    try:
        with pytest.raises(Exception):
            ops.sepconv_fwd(ops.View.plain(x), 1, 8, 16, torch.zeros(9 * 4, device="cuda"), 64,
                            torch.zeros(4 * 64, device="cuda"), None, torch.empty((1, 8, 16, 64), device="cuda"))
    finally:
        ops.sepconv_set_schedule(old)


def test_fused_sepconv_unsupported_shapes(ops):
    x = torch.zeros((1, 8, 8, 16), device="cuda")
    assert not ops.sepconv_supported(ops.View.plain(x), 1, 8, 8, 64)     # w % 16 != 0
    x3 = torch.zeros((1, 16, 16, 3), device="cuda")
    assert not ops.sepconv_supported(ops.View.plain(x3), 1, 16, 16, 64)  # 3 channels


@pytest.mark.parametrize("use_bn", [True, False])
@pytest.mark.parametrize("drop", [0.0, 0.2])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 8, 8, 128, 64), (1, 5, 7, 64, 32), (3, 4, 6, 256, 128),
                                            (2, 16, 16, 128, 128), (4, 64, 144, 128, 64)])  # > 256 slabs
def test_convt_bwd_data_bnstats(ops, use_bn, drop, n, h, w, cin, cout):
    """Conv2DTranspose data gradient that also emits the BN-backward partials of the block below
    (u_net.py:88 upsample fed by a BN+ReLU output; with drop > 0 through the bottleneck's Dropout,
    u_net.py:77-78, so the partials carry the mask): dx bitwise equal to the plain launch,
    statistics equal to unet_bn_relu_bwd_stats's and to float64 numpy."""
    rng = np.random.default_rng(n * 1000 + h * 10 + cin + cout)
    a, t = _view_inputs(rng, 1, n, h, w, cin)
    v = _mk_view(ops, 1, t)
    seed = 4242
    if drop > 0.0:
        v = v.dropout(drop, seed)
    k = dev(f32(rng.standard_normal((2, 2, cout, cin)) * 0.1))
    dout = dev(f32(rng.standard_normal((n, 2 * h, 2 * w, cout))))
    S = ops.conv_transpose2x2_bwd_data_bnstats_slabs(v, n, h, w, cout)
    m = n * h * w
    # one slab per row tile: 64-row tiles when the 128-row grid holds <= 256 blocks of 64 columns
    bm = 64 if (m + 127) // 128 * ((cin + 63) // 64) <= 256 else 128
    assert S == (m + bm - 1) // bm
    mean = dev(f32(rng.standard_normal(cin) * 0.1))
    rstd = dev(f32(1.0 + rng.random(cin)))
    part = torch.zeros(ops.bn_stats_partials_numel(S, cin), device="cuda")  # counters zero
    dx_f, dx_p = torch.empty((n, h, w, cin), device="cuda"), torch.empty((n, h, w, cin), device="cuda")
    ops.conv_transpose2x2_bwd_data_bnstats(v, n, h, w, cout, k, dout, dx_f, mean if use_bn else None,
                                           rstd if use_bn else None, part)
    ops.conv_transpose2x2_bwd(v, n, h, w, cout, k, dout, dx_p, None, None)
    assert torch.equal(dx_f, dx_p)
    outs = []
    for fused in (True, False):
        dg, db, coef = (torch.zeros(cin, device="cuda"), torch.zeros(cin, device="cuda"),
                        torch.empty(3 * cin, device="cuda"))
        if fused:
            ops.bn_relu_bwd_stats_finish(part, S, m, cin, mean, rstd, use_bn, dg if use_bn else None, db, coef)
            assert not torch.any(part[-((cin + 63) // 64):].view(torch.int32))
        else:
            ops.bn_relu_bwd_stats(dx_p, t["src0"], m, cin, mean, rstd, t["sc0"], t["sh0"], use_bn, drop, seed,
                                  dg if use_bn else None, db, coef)
        outs.append((host(dg), host(db), host(coef)))
    for x, y in zip(outs[0], outs[1]):
        assert rel_err(x, y) < 2e-5
    da = host(dx_p).astype(np.float64).reshape(-1, cin)
    if drop > 0.0:  # the documented counter-based mask (oracle/keras_ops.py dropout_mult)
        da = da * K.dropout_mult(seed, (n, h, w, cin), drop).reshape(-1, cin)
    z = a["src0"].astype(np.float64).reshape(-1, cin)
    g = np.where(z * a["sc0"] + a["sh0"] > 0, da, 0.0)
    assert rel_err(outs[0][1], g.sum(0)) < 1e-5
    if use_bn:
        xh = (z - host(mean)) * host(rstd)
        assert rel_err(outs[0][0], (g * xh).sum(0)) < 1e-5


@pytest.mark.parametrize("mode", [2, 1])
@pytest.mark.parametrize("use_bn", [True, False])
@pytest.mark.parametrize("n,h,w,c", [(2, 8, 16, 64), (2, 5, 7, 16), (1, 4, 4, 128), (3, 8, 8, 8),
                                     (4, 64, 144, 64)])  # > 256 slabs: two-pass finish
def test_dwconv_bwd_data_bnstats(ops, mode, use_bn, n, h, w, c):
    """Pool / BN+ReLU-view data gradient that also emits the view block's BN-backward partials:
    dx0 bitwise equal to the plain launch, statistics equal to unet_bn_relu_bwd_stats's."""
    rng = np.random.default_rng(n * 100 + h * 10 + c + mode)
    a, t = _view_inputs(rng, mode, n, h, w, c)
    v = _mk_view(ops, mode, t)
    dk = dev(f32(rng.standard_normal((3, 3, c, 1))))
    dy = dev(f32(rng.standard_normal((n, h, w, c))))
    f = 2 if mode == 2 else 1
    init = f32(rng.standard_normal((n, f * h, f * w, c)))
    S = ops.dwconv3x3_bwd_data_bnstats_slabs(v, n, h, w)
    assert S > 0
    mean = dev(f32(rng.standard_normal(c) * 0.1))
    rstd = dev(f32(1.0 + rng.random(c)))
    part = torch.zeros(ops.bn_stats_partials_numel(S, c), device="cuda")  # counters zero
    dx_f, dx_p = dev(init), dev(init)
    ops.dwconv3x3_bwd_data_bnstats(v, n, h, w, dk, dy, dx_f, mean if use_bn else None, rstd if use_bn else None,
                                   part)
    ops.dwconv3x3_bwd_data(v, n, h, w, dk, dy, dx_p)
    assert torch.equal(dx_f, dx_p)
    m = n * f * f * h * w
    outs = []
    for fused in (True, False):
        dg, db, coef = (torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda"),
                        torch.empty(3 * c, device="cuda"))
        if fused:  # twice: the arrival counters are left zero, the result is deterministic
            ops.bn_relu_bwd_stats_finish(part, S, m, c, mean, rstd, use_bn, dg if use_bn else None, db, coef)
            first = coef.clone()
            ops.bn_relu_bwd_stats_finish(part, S, m, c, mean, rstd, use_bn, dg if use_bn else None, db, coef)
            assert torch.equal(first, coef)
            assert not torch.any(part[-((c + 63) // 64):].view(torch.int32))
        else:
            ops.bn_relu_bwd_stats(dx_p, t["src0"], m, c, mean, rstd, t["sc0"], t["sh0"], use_bn, 0.0, 0,
                                  dg if use_bn else None, db, coef)
        outs.append((host(dg), host(db), host(coef)))
    for x, y in zip(outs[0], outs[1]):
        assert rel_err(x, y) < 2e-5
    # and against float64 numpy: g = da * [z*sc+sh > 0], dbeta = sum g, dgamma = sum g*xhat
    da = host(dx_p).astype(np.float64).reshape(-1, c)
    z = a["src0"].astype(np.float64).reshape(-1, c)
    g = np.where(z * a["sc0"] + a["sh0"] > 0, da, 0.0)
    assert rel_err(outs[0][1], g.sum(0)) < 1e-5
    if use_bn:
        xh = (z - host(mean)) * host(rstd)
        assert rel_err(outs[0][0], (g * xh).sum(0)) < 1e-5


@pytest.mark.parametrize("use_bn", [True, False])
@pytest.mark.parametrize("loss_kind", [0, 1])
@pytest.mark.parametrize("ncls,nhw", [(1, (2, 16, 24)), (21, (2, 16, 24)), (5, (1, 37, 41))])
def test_head_bwd_bnstats(ops, use_bn, loss_kind, ncls, nhw):
    """Head backward that also emits the last block's BN-backward partials (binary, and the fused
    multi-class kernel): dx / dW / db bitwise equal to unet_head_bwd, statistics equal to
    unet_bn_relu_bwd_stats's."""
    rng = np.random.default_rng(11 + loss_kind + ncls)
    n, h, w = nhw
    c = 64
    a, t = _view_inputs(rng, 1, n, h, w, c)
    v = _mk_view(ops, 1, t)
    k = dev(f32(rng.standard_normal((1, 1, c, ncls)) * 0.2))
    if ncls == 1:
        prob = dev(f32(rng.random((n, h, w, 1)) * 0.9 + 0.05))
        yt = dev((rng.random((n, h, w, 1)) > 0.6).astype(np.float32))
    else:
        lg = rng.standard_normal((n, h, w, ncls))
        prob = dev(f32(np.exp(lg) / np.exp(lg).sum(-1, keepdims=True)))
        yt = dev(f32(np.eye(ncls)[rng.integers(0, ncls, (n, h, w))]))
    sums = torch.empty(n * ncls * 3, device="cuda")
    res = torch.empty(3, device="cuda")
    ops.dice_fwd(yt, prob, n, h * w, ncls, 1e-7, sums, res)
    S = ops.head_bwd_bnstats_slabs(v, n, h, w, ncls)
    assert S > 0
    mean = dev(f32(rng.standard_normal(c) * 0.1))
    rstd = dev(f32(1.0 + rng.random(c)))
    part = torch.zeros(ops.bn_stats_partials_numel(S, c), device="cuda")  # counters zero
    outs = []
    for fused in (True, False):
        dx, dk, db = (torch.empty((n, h, w, c), device="cuda"), torch.empty(c * ncls, device="cuda"),
                      torch.empty(ncls, device="cuda"))
        if fused:
            ops.head_bwd_bnstats(v, n, h, w, ncls, k, prob, yt, sums, 1e-7, loss_kind, dx, dk, db,
                                 mean if use_bn else None, rstd if use_bn else None, part)
        else:
            ops.head_bwd(v, n, h, w, ncls, k, prob, yt, sums, 1e-7, loss_kind, dx, dk, db)
        outs.append((dx, dk, db))
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x, y)
    if ncls == 1:
        # rank-one form (ABI 10): only dL/dlogit per pixel goes out; dx == dlogit (x) kernel bitwise,
        # the same weight / bias gradients and BN-backward partials
        dl, dk1, db1 = torch.empty(n * h * w, device="cuda"), torch.empty(c, device="cuda"), torch.empty(1, device="cuda")
        part1 = torch.zeros_like(part)
        ops.head_bwd_bnstats(v, n, h, w, 1, k, prob, yt, sums, 1e-7, loss_kind, None, dk1, db1,
                             mean if use_bn else None, rstd if use_bn else None, part1, dlogit=dl)
        assert torch.equal(dl[:, None] * k.reshape(1, c), outs[0][0].reshape(-1, c))
        assert torch.equal(dk1, outs[0][1]) and torch.equal(db1, outs[0][2])
        assert torch.equal(part1, part)
        with pytest.raises(ValueError):  # neither dx nor dlogit
            ops.head_bwd_bnstats(v, n, h, w, 1, k, prob, yt, sums, 1e-7, loss_kind, None, dk1, db1, None, None, part1)
    m = n * h * w
    st = []
    for fused in (True, False):
        dg, dbb, coef = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda"), torch.empty(3 * c, device="cuda")
        if fused:
            ops.bn_relu_bwd_stats_finish(part, S, m, c, mean, rstd, use_bn, dg if use_bn else None, dbb, coef)
        else:
            ops.bn_relu_bwd_stats(outs[1][0], t["src0"], m, c, mean, rstd, t["sc0"], t["sh0"], use_bn, 0.0, 0,
                                  dg if use_bn else None, dbb, coef)
        st.append((host(dg), host(dbb), host(coef)))
    for x, y in zip(st[0], st[1]):
        assert rel_err(x, y) < 2e-5


def test_copy_strided(ops):
    """Channel padding (3 -> 4, pad channel untouched) and slicing back, bit-exact."""
    x = torch.randn(2, 8, 16, 3, device="cuda")
    xp = torch.full((2, 8, 16, 4), 7.0, device="cuda")
    ops.copy_strided(x, 2 * 8 * 16, 3, 3, xp, 4)
    assert torch.equal(xp[..., :3], x) and bool((xp[..., 3] == 7.0).all())
    back = torch.empty(2, 8, 16, 3, device="cuda")
    ops.copy_strided(xp, 2 * 8 * 16, 3, 4, back, 3)
    assert torch.equal(back, x)
    pk = torch.randn(1, 1, 3, 64, device="cuda")
    pp = torch.zeros(1, 1, 4, 64, device="cuda")
    ops.copy_strided(pk, 1, 3 * 64, 3 * 64, pp, 4 * 64)
    assert torch.equal(pp[:, :, :3], pk) and not pp[:, :, 3].any()
    with pytest.raises(ValueError):
        ops.copy_strided(x, 2 * 8 * 16, 3, 4, xp, 4)  # source too small for its stride


def _pool_ref(a):
    N, H, W, C = a.shape
    return a.reshape(N, H // 2, 2, W // 2, 2, C).max((2, 4))


@pytest.mark.parametrize("n,h,w,c", [(2, 8, 16, 64), (1, 16, 32, 128), (3, 4, 6, 8)])
def test_pool_select(ops, n, h, w, c):
    """unet_pool_select: a BN+ReLU view of the selection reads bitwise the 2x2 max-pool of the BN+ReLU
    view of z (MaxPooling2D, model/u_net.py:69), for gammas of either sign (and +-0) and without BN."""
    rng = np.random.default_rng(n * h + c)
    z = f32(rng.standard_normal((n, h, w, c)) * 2)
    z[0, 0, 0, :4] = z[0, 0, 1, :4]  # ties inside a window
    gamma = f32(rng.standard_normal(c))
    gamma[:2] = [0.0, -0.0]
    rstd = f32(0.5 + rng.random(c))
    scale, shift = f32(gamma * rstd), f32(rng.standard_normal(c) * 0.3)
    out = torch.empty((n, h // 2, w // 2, c), device="cuda")
    for g, sc in ((gamma, scale), (None, np.ones(c, np.float32))):
        ops.pool_select(dev(z), n, h, w, c, None if g is None else dev(g), out)
        tz, tsc, tsh = dev(z), dev(sc), dev(shift)
        got = torch.relu(torch.addcmul(tsh, out, tsc))  # fmaf(sel, sc, sh) as the views evaluate it
        pre = torch.relu(torch.addcmul(tsh, tz, tsc))
        ref = pre.reshape(n, h // 2, 2, w // 2, 2, c).amax((2, 4))
        assert torch.equal(got, ref)


@pytest.mark.parametrize("mode,n,h,w,c0,cout", [(1, 2, 8, 16, 64, 64), (1, 1, 16, 32, 128, 128),
                                                (1, 1, 8, 32, 64, 192), (2, 2, 8, 16, 64, 128)])
def test_sepconv_pool_selection_epilogue(ops, sep_schedule, mode, n, h, w, c0, cout):
    """unet_sepconv_fwd's z_pool_sel (register-A epilogue, or the separate pass after the LDS-A-tile
    kernel) equals unet_pool_select of its own z, bitwise."""
    rng = np.random.default_rng(7 + cout)
    a, t = _view_inputs(rng, mode, n, h, w, c0, 0)
    dk = dev(f32(rng.standard_normal((3, 3, c0, 1))))
    pk = dev(f32(rng.standard_normal((1, 1, c0, cout)) / np.sqrt(c0)))
    v = _mk_view(ops, mode, t)
    gamma = dev(f32(rng.standard_normal(cout)))
    z = torch.empty((n, h, w, cout), device="cuda")
    zsel = torch.full((n, h // 2, w // 2, cout), 7.0, device="cuda")
    ops.sepconv_fwd(v, n, h, w, dk, cout, pk, None, z, None, zsel, gamma)
    ref = torch.empty_like(zsel)
    ops.pool_select(z, n, h, w, cout, gamma, ref)
    assert torch.equal(zsel, ref)


@pytest.mark.parametrize("n,h,w,c0,cout", [(2, 8, 16, 64, 64), (1, 16, 32, 128, 128), (1, 8, 16, 128, 256),
                                           (2, 8, 16, 256, 256), (1, 8, 32, 64, 320)])
def test_sepconv_pool_selection_epilogue_split_precision(ops, n, h, w, c0, cout):
    """The split-precision register-A kernel's pool-selection epilogue (64 / 128 / 256-column
    tiles) equals unet_pool_select of its own z, bitwise."""
    rng = np.random.default_rng(17 + cout)
    a, t = _view_inputs(rng, 1, n, h, w, c0, 0)
    dk = dev(f32(rng.standard_normal((3, 3, c0, 1))))
    pk = dev(f32(rng.standard_normal((1, 1, c0, cout)) / np.sqrt(c0)))
    pkx = torch.empty(3 * c0 * cout, dtype=torch.int16, device="cuda")
    ops.split_x3(pk, [(0, c0, cout, 0)], pkx)
    v = _mk_view(ops, 1, t)
    gamma = dev(f32(rng.standard_normal(cout)))
    z = torch.empty((n, h, w, cout), device="cuda")
    zsel = torch.full((n, h // 2, w // 2, cout), 7.0, device="cuda")
    part = torch.zeros(ops.bn_partials_numel(n * h * w, cout), device="cuda")
    ops.sepconv_fwd(v, n, h, w, dk, cout, pk, None, z, part, zsel, gamma, pkx=pkx)
    ref = torch.empty_like(zsel)
    ops.pool_select(z, n, h, w, cout, gamma, ref)
    assert torch.equal(zsel, ref)
    zr = K.pointwise(K.depthwise3x3(view_value(1, a["src0"], a["sc0"], a["sh0"], None, None, None, 0.0, 0), host(dk)),
                     host(pk))
    assert rel_err(host(z), zr) < 5e-6


@pytest.mark.parametrize("mode,n,h,w,c0,c1,cout,drop", [(1, 2, 8, 16, 64, 0, 64, 0.0), (1, 1, 16, 32, 128, 0, 128, 0.0),
                                                        (3, 1, 16, 16, 64, 64, 64, 0.2), (0, 2, 8, 32, 96, 0, 192, 0.0),
                                                        (1, 1, 8, 16, 256, 0, 256, 0.0),
                                                        # 256-column tiles: two of them, a partial one
                                                        (3, 1, 8, 16, 256, 256, 512, 0.2), (1, 2, 8, 16, 64, 0, 320, 0.0)])
def test_fused_sepconv_split_precision(ops, mode, n, h, w, c0, c1, cout, drop):
    """The register-A kernel's bf16x6 variant (pw_kernel_x3 from unet_split_x3): z within the fp32
    path's tolerance of the float64 oracle, the depthwise output y bitwise equal to the fp32
    variant's (same taps, same fmaf order), BN partials consistent."""
    rng = np.random.default_rng(300 + mode + cout)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk = dev(f32(rng.standard_normal((3, 3, C, 1))))
    pk32 = f32(rng.standard_normal((1, 1, C, cout)) / np.sqrt(C))
    pk = dev(pk32)
    pkx = torch.empty(3 * C * cout, dtype=torch.int16, device="cuda")
    ops.split_x3(pk, [(0, C, cout, 0)], pkx)
    # the planes hold the exact three-way split, transposed
    hm = pkx.view(3, cout, C).cpu().numpy().astype(np.uint16).astype(np.uint32) << 16
    parts = hm.view(np.float32).astype(np.float64)
    assert np.array_equal(parts.sum(0), pk32[0, 0].astype(np.float64).T)
    v = _mk_view(ops, mode, t, drop, 77)
    m = n * h * w
    outs = {}
    for tag, px in (("f32", None), ("x6", pkx)):
        y = torch.full((n, h, w, C), -7.0, device="cuda")
        z = torch.empty((n, h, w, cout), device="cuda")
        part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
        ops.sepconv_fwd(v, n, h, w, dk, cout, pk, y, z, part, pkx=px)
        outs[tag] = (y, z, part)
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"), drop, 77)
    zr = K.pointwise(K.depthwise3x3(xv, host(dk)), pk32)
    assert rel_err(host(outs["x6"][1]), zr) < 5e-6
    assert rel_err(host(outs["x6"][1]), zr) <= 2 * rel_err(host(outs["f32"][1]), zr) + 1e-7
    assert torch.equal(outs["x6"][0], outs["f32"][0])
    assert rel_err(host(outs["x6"][2]), host(outs["f32"][2])) < 1e-5


PX_CASES = [
    # mode, n, h, w, c0, c1, cout, drop, train, zsel
    (1, 2, 8, 16, 64, 0, 128, 0.0, True, True),       # one tile per block
    (1, 3, 64, 96, 64, 0, 128, 0.0, True, False),     # several tiles per block (enc2_block1's shape)
    (1, 7, 88, 208, 128, 0, 128, 0.0, True, True),    # 1001 tiles: runs of 1 and 2 tiles per block
    (3, 2, 32, 64, 64, 64, 64, 0.2, True, False),     # concat + dropout (dec1_block1)
    (3, 1, 16, 32, 64, 64, 128, 0.0, True, False),    # concat, 128 outputs
    (0, 2, 64, 64, 128, 0, 64, 0.0, False, True),     # plain view, 128 -> 64, inference epilogue
    (1, 4, 128, 128, 128, 0, 128, 0.0, True, True),   # enc2_block2's shape at batch 4
    (3, 2, 256, 256, 64, 64, 64, 0.0, True, False),   # dec1_block1's shape at batch 2
    (1, 2, 256, 256, 64, 0, 64, 0.0, True, True),     # enc1_block2's shape (64 -> 64)
]


@pytest.mark.parametrize("mode,n,h,w,c0,c1,cout,drop,train,zsel", PX_CASES)
def test_sepconv_persistent_matches_one_tile(ops, mode, n, h, w, c0, c1, cout, drop, train, zsel):
    """The persistent split-precision forward (sepconv_px.hip, schedule RK: every supported shape)
    against the one-tile-per-block register-A kernel (schedule RK1) with the same split planes: the same
    products in the same order, so z, y and the pooling selection are bitwise equal; the per-tile
    BN partials combine the four waves' 32-row moments by Chan's formula instead of a two-pass sum
    over 128 rows (fp32 rounding apart).  Also against the float64 oracle."""
    rng = np.random.default_rng(900 + mode + n + cout)
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C = c0 + c1
    dk = dev(f32(rng.standard_normal((3, 3, C, 1))))
    pk32 = f32(rng.standard_normal((1, 1, C, cout)) / np.sqrt(C))
    pk = dev(pk32)
    pkx = torch.empty(3 * C * cout, dtype=torch.int16, device="cuda")
    ops.split_x3(pk, [(0, C, cout, 0)], pkx)
    gamma = dev(f32(rng.standard_normal(cout))) if zsel else None
    v = _mk_view(ops, mode, t, drop, 31)
    m = n * h * w
    outs = []
    for sch in (ops.SEPCONV_RK1, ops.SEPCONV_RK):
        old = ops.sepconv_set_schedule(sch)
        try:
            y = torch.full((n, h, w, C), -7.0, device="cuda") if train else None
            z = torch.full((n, h, w, cout), float("nan"), device="cuda")
            part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda") if train else None
            zs = torch.full((n, h // 2, w // 2, cout), float("nan"), device="cuda") if zsel else None
            ops.sepconv_fwd(v, n, h, w, dk, cout, pk, y, z, part, zs, gamma, pkx=pkx)
            torch.cuda.synchronize()
            outs.append([None if q is None else q.cpu() for q in (y, z, part, zs)])
        finally:
            ops.sepconv_set_schedule(old)
    (y1, z1, p1, s1), (y2, z2, p2, s2) = outs
    assert torch.equal(z1, z2)
    if train:
        assert torch.equal(y1, y2)
        nb = m // 128 * cout * 2
        pa, pb = p1[:nb].view(-1, cout, 2).double(), p2[:nb].view(-1, cout, 2).double()
        assert float((pa[..., 0] - pb[..., 0]).abs().max()) <= 1e-6 * float(pa[..., 0].abs().max() + 1)
        assert rel_err(pb[..., 1].numpy(), pa[..., 1].numpy()) < 1e-5
    if zsel:
        assert torch.equal(s1, s2)
    if m <= 64 * 1024:
        xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"), drop, 31)
        zr = K.pointwise(K.depthwise3x3(xv, host(dk)), pk32)
        assert rel_err(z2.numpy(), zr) < 5e-6


@pytest.mark.parametrize("mode,n,h,w,c0,c1", [(1, 2, 8, 16, 64, 0), (1, 1, 16, 32, 64, 0), (3, 1, 8, 32, 64, 64),
                                              (0, 2, 16, 16, 128, 0)])
@pytest.mark.parametrize("use_bn", [True, False])
def test_sepconv_bwd_fused(ops, mode, n, h, w, c0, c1, use_bn):
    """The fused 64-output block backward (unet_sepconv_bwd_fused) against the route it replaces:
    unet_pointwise_bwd_data_bnrelu (dz formed on load, dy) + unet_sepconv_bwd_filter over that dz /
    dy, and against the float64 oracle's BN + ReLU backward and weight gradients."""
    rng = np.random.default_rng(700 + mode + n + (7 if use_bn else 0))
    a, t = _view_inputs(rng, mode, n, h, w, c0, c1)
    C, cout, m = c0 + c1, 64, n * h * w
    dk = dev(f32(rng.standard_normal((3, 3, C, 1))))
    pk32 = f32(rng.standard_normal((1, 1, C, cout)) / np.sqrt(C))
    pk = dev(pk32)
    z = f32(rng.standard_normal((m, 1, 1, cout)) * 2 + 0.3)
    da = f32(rng.standard_normal((m, 1, 1, cout)))
    gamma, beta = bn_affine(rng, cout)
    if use_bn:
        _, mean, var = K.bn_train(z, gamma, beta)
        rstd = 1 / np.sqrt(var + 1e-3)
        scale, shift = f32(gamma * rstd), f32(beta - mean * gamma * rstd)
    else:
        mean = var = rstd = np.zeros(cout)
        scale, shift = np.ones(cout, np.float32), f32(beta)
    ts, th, tz, tda = dev(scale), dev(shift), dev(z), dev(da)
    coef = torch.empty(3 * cout, device="cuda")
    dg, db = torch.zeros(cout, device="cuda"), torch.zeros(cout, device="cuda")
    ops.bn_relu_bwd_stats(tda, tz, m, cout, dev(f32(mean)), dev(f32(rstd)), ts, th, use_bn, 0.0, 0,
                          dg if use_bn else None, db, coef)
    v = _mk_view(ops, mode, t)
    dy_f = torch.full((n, h, w, C), 7.0, device="cuda")
    ddk_f, dpk_f = torch.empty((3, 3, C, 1), device="cuda"), torch.empty((1, 1, C, cout), device="cuda")
    ops.sepconv_bwd_fused(v, n, h, w, dk, pk, tda, tz, ts, th, coef, cout, dy_f, ddk_f, dpk_f)
    dy_r, dz_r = torch.empty((m, C), device="cuda"), torch.empty((m, cout), device="cuda")
    ops.pointwise_bwd_data_bnrelu(tda, tz, m, C, cout, pk, ts, th, coef, 0.0, 0, dy_r, dz_r)
    ddk_r, dpk_r = torch.empty((3, 3, C, 1), device="cuda"), torch.empty((1, 1, C, cout), device="cuda")
    ops.sepconv_bwd_filter(v, n, h, w, dk, dy_r, dz_r, cout, ddk_r, dpk_r)
    assert rel_err(host(dy_f).reshape(m, C), host(dy_r)) < 2e-6
    assert rel_err(host(dpk_f), host(dpk_r)) < 2e-6
    assert rel_err(host(ddk_f), host(ddk_r)) < 2e-6
    # the binary head's rank-one da (ABI 10): da = dlogit (x) kernel formed on load, bitwise the same
    dlg = dev(f32(rng.standard_normal(m)))
    hk = dev(f32(rng.standard_normal(cout) * 0.3))
    da1 = dlg[:, None] * hk[None, :]
    outs1 = []
    for r1 in (False, True):
        dy1 = torch.full((n, h, w, C), 7.0, device="cuda")
        ddk1, dpk1 = torch.empty((3, 3, C, 1), device="cuda"), torch.empty((1, 1, C, cout), device="cuda")
        if r1:
            ops.sepconv_bwd_fused(v, n, h, w, dk, pk, None, tz, ts, th, coef, cout, dy1, ddk1, dpk1, da_rank1=(dlg, hk))
        else:
            ops.sepconv_bwd_fused(v, n, h, w, dk, pk, da1, tz, ts, th, coef, cout, dy1, ddk1, dpk1)
        outs1.append((dy1, ddk1, dpk1))
    for x1, x2 in zip(*outs1):
        assert torch.equal(x1, x2)
    # float64 oracle
    if use_bn:
        rz, _, _ = K.bn_relu_bwd(da, z, gamma, beta, f32(mean), f32(var))
    else:
        rz = np.where(z + beta > 0, da, 0)
    rz = rz.reshape(m, cout).astype(np.float64)
    ry = rz @ pk32[0, 0].T.astype(np.float64)
    assert rel_err(host(dy_f).reshape(m, C), ry) < 1e-4
    xv = view_value(mode, a["src0"], a.get("sc0"), a.get("sh0"), a.get("src1"), a.get("sc1"), a.get("sh1"),
                    0.0, 0).astype(np.float64)
    yr = K.depthwise3x3(xv, host(dk).astype(np.float64))
    assert rel_err(host(dpk_f).reshape(C, cout), yr.reshape(m, C).T @ rz) < 1e-4
