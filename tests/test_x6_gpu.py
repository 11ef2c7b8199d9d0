"""Split-precision (bf16x6) rows-GEMM routes of ABI 12 against the float64 oracle: the BatchNorm-
backward data gradient (unet_pointwise_bwd_data_bnrelu_x3), the Conv2DTranspose forward
(unet_conv_transpose2x2_fwd_x3) and its data gradient with BN partials
(unet_conv_transpose2x2_bwd_data_bnstats_x3), with the weight planes from unet_split_x3_keep /
unet_split_x3.  Shapes include ragged pixel counts (not a multiple of the 128-row tile), column
counts that are not a multiple of the 128-column tile, dropout, and k depths that are not a
multiple of 32 (those take the fp32 route and must equal it bitwise).

Reference: model/u_net.py:14-25 (SeparableConv2D pointwise -> BatchNormalization -> ReLU),
u_net.py:88-94 (Conv2DTranspose); the six-product split is common.h split4 / mfma_x6."""
import numpy as np
import pytest

from helpers import bn_affine, dev, f32, host, rel_err
from oracle import keras_ops as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# fp32-accurate: the six significant bf16 part products drop terms of ~2^-23 |a b|, below the fp32
# accumulation's own rounding; the fp32-MFMA route measures 1.4e-7 ... 6e-7 on these shapes (the
# 2048-deep ConvT data gradient 2.2e-6: there the bar is 1.5 x the fp32 route's own distance)
TOL = 2e-6


@pytest.fixture(scope="module")
def ops():
    from unet_amd import ops as O
    return O


def _planes(ops, w2d: np.ndarray, keep: bool):
    rows, cols = w2d.shape
    t = torch.empty(3 * rows * cols, dtype=torch.int16, device="cuda")
    ops.split_x3(dev(f32(w2d)), [(0, rows, cols, 0)], t, keep=keep)
    return t


def _tiles(m: int, n: int) -> int:
    """128 x 128 tiles of an (m, n) output: the split-precision route needs >= 256 of them and n > 64
    (gemm.hip rows_x6)"""
    return 0 if n <= 64 else (m + 127) // 128 * ((n + 127) // 128)


def _bf16(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint16).astype(np.uint32) << 16).view(np.float32)


@pytest.mark.parametrize("keep", [False, True])
@pytest.mark.parametrize("rows,cols", [(64, 96), (37, 5), (512, 256)])
def test_split_x3_exact(ops, keep, rows, cols):
    """hi + mid + lo == w exactly (float64 sum of the three bf16 planes), in either layout."""
    rng = np.random.default_rng(rows + 7 * cols + keep)
    w = f32(rng.standard_normal((rows, cols)) * np.exp(rng.uniform(-8, 8, (rows, cols))))
    t = host(_planes(ops, w, keep)).reshape(3, -1)
    p = [_bf16(t[i]).astype(np.float64) for i in range(3)]
    s = (p[0] + p[1] + p[2]).reshape((rows, cols) if keep else (cols, rows))
    np.testing.assert_array_equal(s if keep else s.T, w.astype(np.float64))


def _bnbwd_case(rng, m, cout, use_bn=True):
    z = f32(rng.standard_normal((m, cout)) * 2 + 0.3)
    da = f32(rng.standard_normal((m, cout)))
    gamma, beta = bn_affine(rng, cout)
    mean, var = z.astype(np.float64).mean(0), z.astype(np.float64).var(0)
    rstd = 1 / np.sqrt(var + 1e-3)
    scale, shift = f32(gamma * rstd), f32(beta - mean * gamma * rstd)
    return z, da, f32(mean), f32(rstd), scale, shift


@pytest.mark.parametrize("drop", [0.0, 0.2])
@pytest.mark.parametrize("m,cin,cout", [(33000, 96, 128), (16384, 256, 256), (33000, 512, 64), (33000, 128, 1024),
                                        (33000, 64, 48), (4096, 512, 256), (33000, 64, 128), (40000, 40, 64)])
def test_pointwise_bwd_data_bnrelu_x3(ops, drop, m, cin, cout):
    """dy = dz . pk^T with dz formed on load: the split-precision route within TOL of float64 of the
    same dz; cout = 1024 takes the streaming-dz route + the plain split-precision GEMM; cout = 48 (k
    not a multiple of 32) and 4096 x 256 (a grid of < 256 tiles) take the fp32 route, bitwise."""
    rng = np.random.default_rng(m + cin + cout + int(10 * drop))
    z, da, mean, rstd, scale, shift = _bnbwd_case(rng, m, cout)
    pk = f32(rng.standard_normal((cin, cout)) / np.sqrt(cout))
    pkd = _planes(ops, pk, keep=True)
    ts, th = dev(scale), dev(shift)
    dg, db, coef = torch.zeros(cout, device="cuda"), torch.zeros(cout, device="cuda"), torch.empty(3 * cout, device="cuda")
    ops.bn_relu_bwd_stats(dev(da), dev(z), m, cout, dev(mean), dev(rstd), ts, th, True, drop, 55, dg, db, coef)
    out = {}
    for key in ("f32", "x6"):
        dy = torch.full((m, cin), 7.0, device="cuda")
        dz = torch.full((m, cout), 7.0, device="cuda")
        ops.pointwise_bwd_data_bnrelu(dev(da), dev(z), m, cin, cout, dev(pk), ts, th, coef, drop, 55, dy, dz,
                                      pkd=pkd if key == "x6" else None)
        out[key] = (host(dy), host(dz))
    # the same dz expression in both instantiations (fp contraction may differ by an ulp)
    assert rel_err(out["x6"][1], out["f32"][1].astype(np.float64)) < 1e-6
    ref = out["x6"][1].astype(np.float64) @ pk.astype(np.float64).T
    assert rel_err(out["x6"][0], ref) < TOL
    if cout % 32 or _tiles(m, cin) < 256:
        assert np.array_equal(out["f32"][0], out["x6"][0])  # (fp32 route taken)
    # the formed dz itself against the oracle's BN + ReLU (+ dropout) backward
    dmult = K.dropout_mult(55, (m, 1, 1, cout), drop).reshape(m, cout) if drop > 0 else None
    g = da if dmult is None else da * dmult
    g = np.where(z * scale + shift > 0, g, 0).astype(np.float64)
    rz = scale * (g - g.mean(0) - (z - mean) * rstd * (g * (z - mean) * rstd).mean(0))
    assert rel_err(out["x6"][1], rz) < 1e-4


@pytest.mark.parametrize("stats", [False, True])
@pytest.mark.parametrize("m,cin,cout", [(33000, 96, 160), (16384, 512, 1024), (4096, 256, 256), (200, 48, 64)])
def test_pointwise_fwd_x3(ops, stats, m, cin, cout):
    """Pointwise forward (the bottleneck's split route) with the BN-statistics epilogue through the
    split-precision route: z within TOL of float64, per-tile (mean, M2) partials within 1e-5 of the
    fp32 route's (they summarise the route's own z); cin = 48 equals the fp32 route bitwise."""
    rng = np.random.default_rng(m + cin + cout + stats)
    y = f32(rng.standard_normal((m, cin)))
    pk = f32(rng.standard_normal((cin, cout)) / np.sqrt(cin))
    pkx = _planes(ops, pk, keep=False)
    res = {}
    for key in ("f32", "x6"):
        z = torch.full((m, cout), 7.0, device="cuda")
        part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda") if stats else None
        ops.pointwise_fwd(dev(y), m, cin, cout, dev(pk), z, part, pkx=pkx if key == "x6" else None)
        res[key] = (host(z), host(part) if stats else None)
    ref = y.astype(np.float64) @ pk.astype(np.float64)
    assert rel_err(res["x6"][0], ref) < TOL
    if stats:
        assert rel_err(res["x6"][1], res["f32"][1]) < 1e-5
    if cin % 32 or _tiles(m, cout) < 256:
        assert np.array_equal(res["f32"][0], res["x6"][0])


@pytest.mark.parametrize("drop", [0.0, 0.2])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 130, 127, 64, 32), (4, 64, 64, 256, 128), (13, 33, 41, 96, 40),
                                            (1, 4, 4, 1024, 512), (2, 6, 6, 48, 16)])
def test_conv_transpose_fwd_x3(ops, drop, n, h, w, cin, cout):
    """Conv2DTranspose forward (BN+ReLU view, dropout as at the bottleneck) through the split-
    precision route against float64; cin = 48 (k not a multiple of 32) equals the fp32 route."""
    rng = np.random.default_rng(n * h * w + cin + cout)
    z = f32(rng.standard_normal((n, h, w, cin)))
    sc, sh = bn_affine(rng, cin)
    v = ops.View.bnrelu(dev(z), dev(sc), dev(sh))
    if drop > 0:
        v = v.dropout(drop, 4242)
    x = np.maximum(z * sc + sh, 0)
    if drop > 0:
        x = x * K.dropout_mult(4242, x.shape, drop)
    k = f32(rng.standard_normal((2, 2, cout, cin)) / np.sqrt(cin))
    b = f32(rng.standard_normal(cout))
    kx = _planes(ops, k.reshape(4 * cout, cin), keep=True)
    out = {}
    for key in ("f32", "x6"):
        o = torch.full((n, 2 * h, 2 * w, cout), 7.0, device="cuda")
        ops.conv_transpose2x2_fwd(v, n, h, w, cout, dev(k), dev(b), o, kx=kx if key == "x6" else None)
        out[key] = host(o)
    ref = K.conv_transpose2x2(x.astype(np.float64), k, b)
    assert rel_err(out["x6"], ref) < TOL
    if cin % 32 or _tiles(n * h * w, 4 * cout) < 256:
        assert np.array_equal(out["f32"], out["x6"])


@pytest.mark.parametrize("drop", [0.0, 0.2])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 130, 127, 64, 32), (16, 32, 32, 256, 128), (1, 8, 8, 1024, 512),
                                            (2, 6, 6, 48, 20)])
def test_convt_bwd_data_bnstats_x3(ops, drop, n, h, w, cin, cout):
    """Conv2DTranspose data gradient + the BN-backward partials of the block below, split-precision
    route: dx within TOL of float64, the finished statistics equal to the fp32 route's within 1e-5
    (the partials sum the route's own dx)."""
    rng = np.random.default_rng(n * 1000 + h * 10 + cin + cout)
    z = f32(rng.standard_normal((n, h, w, cin)))
    sc, sh = bn_affine(rng, cin)
    v = ops.View.bnrelu(dev(z), dev(sc), dev(sh))
    if drop > 0:
        v = v.dropout(drop, 4242)
    k = f32(rng.standard_normal((2, 2, cout, cin)) * 0.1)
    kxt = _planes(ops, k.reshape(4 * cout, cin), keep=False)
    dout = f32(rng.standard_normal((n, 2 * h, 2 * w, cout)))
    S = ops.conv_transpose2x2_bwd_data_bnstats_slabs(v, n, h, w, cout)
    mean = dev(f32(rng.standard_normal(cin) * 0.1))
    rstd = dev(f32(1.0 + rng.random(cin)))
    m = n * h * w
    res = {}
    for key in ("f32", "x6"):
        part = torch.zeros(ops.bn_stats_partials_numel(S, cin), device="cuda")
        dx = torch.full((n, h, w, cin), 7.0, device="cuda")
        ops.conv_transpose2x2_bwd_data_bnstats(v, n, h, w, cout, dev(k), dev(dout), dx, mean, rstd, part,
                                               kxt=kxt if key == "x6" else None)
        dg, db, coef = torch.zeros(cin, device="cuda"), torch.zeros(cin, device="cuda"), torch.empty(3 * cin,
                                                                                                     device="cuda")
        ops.bn_relu_bwd_stats_finish(part, S, m, cin, mean, rstd, True, dg, db, coef)
        res[key] = (host(dx), host(dg), host(db))
    ref = np.einsum("niajbd,abdc->nijc", dout.astype(np.float64).reshape(n, h, 2, w, 2, cout), k.astype(np.float64))
    assert rel_err(res["x6"][0], ref) < max(TOL, 1.5 * rel_err(res["f32"][0], ref))
    assert rel_err(res["x6"][1], res["f32"][1]) < 1e-5
    assert rel_err(res["x6"][2], res["f32"][2]) < 1e-5
    if (4 * cout) % 32 or _tiles(m, cin) < 256 or (m + 127) // 128 * ((cin + 63) // 64) <= 256:
        assert np.array_equal(res["f32"][0], res["x6"][0])


@pytest.mark.parametrize("m,cin,cout", [(33000, 128, 128), (65536, 256, 512), (4100, 96, 200), (1000, 64, 128)])
def test_pointwise_bwd_filter_x6(ops, m, cin, cout):
    """Pointwise weight gradient dW = y^T dz: 128 x 128 output tiles take the split-precision kernel
    (both operands split as they are staged, 32-pixel stages), 64-wide tiles the fp32 one; within
    TOL (or 1.5 x the fp32 float32-sum bound) of float64, ragged pixel counts and column tiles."""
    rng = np.random.default_rng(m + cin + cout)
    y = f32(rng.standard_normal((m, cin)))
    dz = f32(rng.standard_normal((m, cout)))
    dpk = torch.full((cin, cout), 7.0, device="cuda")
    ops.pointwise_bwd_filter(dev(y), dev(dz), m, cin, cout, dpk)
    ref = y.astype(np.float64).T @ dz.astype(np.float64)
    assert rel_err(host(dpk), ref) < TOL


@pytest.mark.parametrize("drop", [0.0, 0.2])
@pytest.mark.parametrize("n,h,w,cin,cout", [(4, 32, 32, 256, 128), (2, 33, 17, 96, 40), (16, 16, 16, 512, 256)])
def test_conv_transpose_bwd_filter_x6(ops, drop, n, h, w, cin, cout):
    """Conv2DTranspose kernel + bias gradients (the split-precision weight-gradient kernel on its
    128 x 128 tiles, the bias as the column sums its q-tile-0 blocks take of dU') against float64."""
    rng = np.random.default_rng(n * h * w + cin + cout)
    z = f32(rng.standard_normal((n, h, w, cin)))
    sc, sh = bn_affine(rng, cin)
    v = ops.View.bnrelu(dev(z), dev(sc), dev(sh))
    x = np.maximum(z * sc + sh, 0).astype(np.float64)
    if drop > 0:
        v = v.dropout(drop, 4242)
        x = x * K.dropout_mult(4242, x.shape, drop)
    k = f32(rng.standard_normal((2, 2, cout, cin)) * 0.1)
    dout = f32(rng.standard_normal((n, 2 * h, 2 * w, cout)))
    dk = torch.full((2, 2, cout, cin), 7.0, device="cuda")
    db = torch.full((cout,), 7.0, device="cuda")
    ops.conv_transpose2x2_bwd(v, n, h, w, cout, dev(k), dev(dout), None, dk, db)
    d6 = dout.astype(np.float64).reshape(n, h, 2, w, 2, cout)
    rdk = np.einsum("niajbd,nijc->abdc", d6, x)
    assert rel_err(host(dk), rdk) < TOL
    assert rel_err(host(db), d6.sum((0, 1, 2, 3, 4))) < 1e-5


def test_split_x3_mixed(ops):
    """One mixed-layout launch (unet_split_x3_mixed, the train step's per-forward refresh) writes the
    same planes as the two single-layout launches."""
    rng = np.random.default_rng(77)
    src = dev(f32(rng.standard_normal(5000)))
    segs = [(0, 40, 30, 0, 1), (1200, 16, 48, 3600, 0), (2000, 33, 17, 6000, 1)]
    mixed = torch.zeros(8000, dtype=torch.int16, device="cuda")
    ops.split_x3(src, segs, mixed)
    ref = torch.zeros(8000, dtype=torch.int16, device="cuda")
    for so, r, c, do, k in segs:
        ops.split_x3(src, [(so, r, c, do)], ref, keep=bool(k))
    assert torch.equal(mixed, ref)
