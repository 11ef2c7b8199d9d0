"""Lab: the decoder block1 forwards (CONCAT view [up | BN+ReLU(skip)], training: y stored where the
step stores it, BN statistics) at configs[1]'s batch 16, with and without the dropout that
u_net.py:97-98 puts on dec4..dec2's concat, each timed with HIP events around 10 back-to-back
launches (median of 3 groups), against the stream floor of the same bytes (t = bytes / 5.3 TB/s).
usage: python tools/lab_dec.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch

from unet_amd import ops
from unet_amd.ops import View

B = int(os.environ.get("B", 16))
g = torch.Generator(device="cpu").manual_seed(7)
dev = "cuda"


def rnd(*s):
    return (torch.rand(s, generator=g) * 2 - 1).to(dev)


def case(name, hw, cu, cs, cout, y_store, drop):
    up, skip = rnd(B, hw, hw, cu), rnd(B, hw, hw, cs)
    sc, sh = rnd(cs) + 1.5, rnd(cs) * 0.1
    cin = cu + cs
    dk, pk = rnd(3, 3, cin, 1), rnd(1, 1, cin, cout) * 0.1
    pkx = torch.empty(3 * cin * cout, dtype=torch.int16, device=dev)
    ops.split_x3(pk, [(0, cin, cout, 0)], pkx)
    m = B * hw * hw
    z = torch.empty(B, hw, hw, cout, device=dev)
    y = torch.empty(B, hw, hw, cin, device=dev) if y_store else None
    part = torch.zeros(ops.bn_partials_numel(m, cout), device=dev)
    v = View.concat(up, skip, sc, sh)
    if drop:
        v = v.dropout(0.2, 12345)
    fn = lambda: ops.sepconv_fwd(v, B, hw, hw, dk, cout, pk, y, z, part, None, None, pkx)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 100)
    us = sorted(ts)[1]
    byts = 4.0 * m * (cin + cout + (cin if y_store else 0))
    print(json.dumps({"block": name, "drop": drop, "us": round(us, 1), "MB": round(byts / 1e6),
                      "floor_us_5.3TBs": round(byts / 5.3e6, 1), "frac_floor": round(byts / 5.3e6 / us, 3)}), flush=True)


for drop in (False, True):
    case("dec3_block1", 64, 256, 256, 256, True, drop)
    case("dec2_block1", 128, 128, 128, 128, True, drop)
    case("dec1_block1", 256, 64, 64, 64, False, drop)
