"""Rows GEMMs, fp32-MFMA route vs the split-precision (bf16x6) route (round 6) per train-step shape
at configs[1] (batch 16): the BatchNorm-backward data gradient (unet_pointwise_bwd_data_bnrelu_x3:
time per launch, accuracy of dy against a float64 product of the same dz, dz equality), the
Conv2DTranspose forward (_fwd_x3) and its data gradient with BN partials (_bwd_data_bnstats_x3).

    python tools/bench_dgrad_x6.py [TAG]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch  # noqa: E402
from unet_amd import ops  # noqa: E402
from unet_amd.ops import View  # noqa: E402

PEAK = 157.3
B = int(os.environ.get("B", 16))
DROP = float(os.environ.get("DROP", 0.0))
TAG = sys.argv[1] if len(sys.argv) > 1 else "x6"
DGRAD = [("enc2_block1", 128, 64, 128), ("enc2_block2", 128, 128, 128), ("enc3_block1", 64, 128, 256), ("enc3_block2", 64, 256, 256),
         ("enc4_block1", 32, 256, 512), ("enc4_block2", 32, 512, 512), ("bneck_block1", 16, 512, 1024),
         ("dec4_block2", 32, 512, 512), ("dec3_block1", 64, 512, 256), ("dec3_block2", 64, 256, 256),
         ("dec2_block1", 128, 256, 128), ("dec2_block2", 128, 128, 128)]
CONVT = [("dec4_upsample", 16, 1024, 512), ("dec3_upsample", 32, 512, 256), ("dec2_upsample", 64, 256, 128),
         ("dec1_upsample", 128, 128, 64)]


def bench(fn, iters=int(os.environ.get("ITERS", 20))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def rel(a, b):
    return float((a.double() - b).norm() / b.norm())


def main():
    g = torch.Generator(device="cpu").manual_seed(3)
    tot = {"f32": 0.0, "x6": 0.0}
    for name, hw, cin, cout in DGRAD:
        m = B * hw * hw
        da = torch.randn(m, cout, generator=g).to("cuda")
        z = torch.randn(m, cout, generator=g).to("cuda")
        pk = (torch.randn(cin, cout, generator=g) / cin ** 0.5).to("cuda")
        pkd = torch.empty(3 * cin * cout, dtype=torch.int16, device="cuda")
        ops.split_x3(pk, [(0, cin, cout, 0)], pkd, keep=True)
        sc = (torch.rand(cout, generator=g) + 0.5).to("cuda")
        sh = (torch.randn(cout, generator=g) * 0.1).to("cuda")
        coef = (torch.randn(3 * cout, generator=g) * 0.1).to("cuda")
        dy = {k: torch.empty(m, cin, device="cuda") for k in tot}
        dz = {k: torch.empty(m, cout, device="cuda") for k in tot}
        fl = 2.0 * m * cin * cout
        res = {}
        for k in tot:
            kw = {"pkd": pkd} if k == "x6" else {}
            s = bench(lambda: ops.pointwise_bwd_data_bnrelu(da, z, m, cin, cout, pk, sc, sh, coef, DROP, 7, dy[k],
                                                            dz[k], **kw))
            tot[k] += s
            res[k] = s
        ref = dz["f32"].double() @ pk.double().T
        out = {"tag": TAG, "block": name, "m": m, "k": cout, "n": cin, "drop": DROP,
               "us_f32": round(res["f32"] * 1e6, 1), "us_x6": round(res["x6"] * 1e6, 1),
               "frac_f32": round(fl / res["f32"] / 1e12 / PEAK, 3), "frac_x6": round(fl / res["x6"] / 1e12 / PEAK, 3),
               "rel_f32": rel(dy["f32"], ref), "rel_x6": rel(dy["x6"], ref),
               "dz_equal": bool(torch.equal(dz["f32"], dz["x6"]))}
        print(json.dumps(out), flush=True)
        del da, z, dy, dz
    print(json.dumps({"tag": TAG, "op": "dgrad", "total_us_f32": round(tot["f32"] * 1e6, 1),
                      "total_us_x6": round(tot["x6"] * 1e6, 1)}), flush=True)
    tot = {"f32": 0.0, "x6": 0.0}
    for name, hw, cin, cout in [("bneck_block1", 16, 512, 1024), ("bneck_block2", 16, 1024, 1024),
                                ("enc4_block2", 32, 512, 512)]:
        m = B * hw * hw
        fl = 2.0 * m * cin * cout
        y = torch.randn(m, cin, generator=g).to("cuda")
        pk = (torch.randn(cin, cout, generator=g) / cin ** 0.5).to("cuda")
        pkx = torch.empty(3 * cin * cout, dtype=torch.int16, device="cuda")
        ops.split_x3(pk, [(0, cin, cout, 0)], pkx)
        part = torch.zeros(ops.bn_partials_numel(m, cout), device="cuda")
        res, outs = {}, {}
        for key in tot:
            outs[key] = torch.empty(m, cout, device="cuda")
            kw = {"pkx": pkx} if key == "x6" else {}
            res[key] = bench(lambda: ops.pointwise_fwd(y, m, cin, cout, pk, outs[key], part, **kw))
            tot[key] += res[key]
        ref = y.double() @ pk.double()
        print(json.dumps({"tag": TAG, "op": "pointwise_fwd", "block": name, "m": m, "k": cin, "n": cout,
                          "us_f32": round(res["f32"] * 1e6, 1), "us_x6": round(res["x6"] * 1e6, 1),
                          "frac_f32": round(fl / res["f32"] / 1e12 / PEAK, 3),
                          "frac_x6": round(fl / res["x6"] / 1e12 / PEAK, 3),
                          "rel_f32": rel(outs["f32"], ref), "rel_x6": rel(outs["x6"], ref)}), flush=True)
    print(json.dumps({"tag": TAG, "op": "pointwise_fwd", "total_us_f32": round(tot["f32"] * 1e6, 1),
                      "total_us_x6": round(tot["x6"] * 1e6, 1)}), flush=True)
    for op in ("convT_fwd", "convT_bwd_data_bnstats"):
        tot = {"f32": 0.0, "x6": 0.0}
        for name, hw, cin, cout in CONVT:
            m = B * hw * hw
            fl = 8.0 * m * cin * cout
            k = (torch.randn(2, 2, cout, cin, generator=g) / cin ** 0.5).to("cuda")
            kx = torch.empty(3 * k.numel(), dtype=torch.int16, device="cuda")
            ops.split_x3(k, [(0, 4 * cout, cin, 0)], kx, keep=(op == "convT_fwd"))
            res, outs = {}, {}
            if op == "convT_fwd":
                z = torch.randn(B, hw, hw, cin, generator=g).to("cuda")
                sc = (torch.rand(cin, generator=g) + 0.5).to("cuda")
                sh = (torch.randn(cin, generator=g) * 0.1).to("cuda")
                v = View.bnrelu(z, sc, sh)
                b = torch.randn(cout, generator=g).to("cuda")
                xin = torch.relu(z.double() * sc.double() + sh.double())
                ref = torch.einsum("nijc,abdc->niajbd", xin, k.double()).reshape(B, 2 * hw, 2 * hw, cout) + b.double()
                for key in tot:
                    outs[key] = torch.empty(B, 2 * hw, 2 * hw, cout, device="cuda")
                    kw = {"kx": kx} if key == "x6" else {}
                    res[key] = bench(lambda: ops.conv_transpose2x2_fwd(v, B, hw, hw, cout, k, b, outs[key], **kw))
            else:
                z = torch.randn(B, hw, hw, cin, generator=g).to("cuda")
                sc = (torch.rand(cin, generator=g) + 0.5).to("cuda")
                sh = (torch.randn(cin, generator=g) * 0.1).to("cuda")
                v = View.bnrelu(z, sc, sh)
                dout = torch.randn(B, 2 * hw, 2 * hw, cout, generator=g).to("cuda")
                mu = torch.randn(cin, generator=g).to("cuda")
                rs = (torch.rand(cin, generator=g) + 0.5).to("cuda")
                S = ops.conv_transpose2x2_bwd_data_bnstats_slabs(v, B, hw, hw, cout)
                ref = torch.einsum("niajbd,abdc->nijc", dout.double().reshape(B, hw, 2, hw, 2, cout), k.double())
                parts = {}
                for key in tot:
                    outs[key] = torch.empty(B, hw, hw, cin, device="cuda")
                    parts[key] = torch.zeros(ops.bn_stats_partials_numel(S, cin), device="cuda")
                    kw = {"kxt": kx} if key == "x6" else {}
                    res[key] = bench(lambda: ops.conv_transpose2x2_bwd_data_bnstats(
                        v, B, hw, hw, cout, k, dout, outs[key], mu, rs, parts[key], **kw))
            for key in tot:
                tot[key] += res[key]
            print(json.dumps({"tag": TAG, "op": op, "block": name, "m": m, "k": cin, "n": cout,
                              "us_f32": round(res["f32"] * 1e6, 1), "us_x6": round(res["x6"] * 1e6, 1),
                              "frac_f32": round(fl / res["f32"] / 1e12 / PEAK, 3),
                              "frac_x6": round(fl / res["x6"] / 1e12 / PEAK, 3),
                              "rel_f32": rel(outs["f32"], ref), "rel_x6": rel(outs["x6"], ref)}), flush=True)
        print(json.dumps({"tag": TAG, "op": op, "total_us_f32": round(tot["f32"] * 1e6, 1),
                          "total_us_x6": round(tot["x6"] * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
