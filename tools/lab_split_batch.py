"""Lab: does splitting a forward op's batch into two halves on two HIP streams (joined after every
op, as a per-block BatchNorm finalize would need) beat the one full-batch launch?  Times 10
back-to-back ops each way (median of 3 groups) on the train step's forward shapes at batch 16.
usage: python tools/lab_split_batch.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch

from unet_amd import ops
from unet_amd.ops import View

B = 16
g = torch.Generator(device="cpu").manual_seed(5)
dev = "cuda"


def rnd(*s):
    return (torch.rand(s, generator=g) * 2 - 1).to(dev)


def sep_case(hw, cin, cout, sel):
    x = rnd(B, hw, hw, cin)
    sc, sh = rnd(cin) + 1.5, rnd(cin) * 0.1
    dk, pk = rnd(3, 3, cin, 1), rnd(1, 1, cin, cout) * 0.1
    pkx = torch.empty(3 * cin * cout, dtype=torch.int16, device=dev)
    ops.split_x3(pk, [(0, cin, cout, 0)], pkx)
    z = torch.empty(B, hw, hw, cout, device=dev)
    y = torch.empty(B, hw, hw, cin, device=dev)
    part = torch.zeros(ops.bn_partials_numel(B * hw * hw, cout), device=dev)
    zs = torch.empty(B, hw // 2, hw // 2, cout, device=dev) if sel else None
    gam = rnd(cout) if sel else None
    h = B // 2
    tiles_half = h * hw * hw // 128

    def run(lo, n):
        v = View.bnrelu(x[lo:lo + n], sc, sh)
        m = n * hw * hw
        ops.sepconv_fwd(v, n, hw, hw, dk, cout, pk, y[lo:lo + n] if cin >= 128 else None, z[lo:lo + n],
                        part[(lo * hw * hw // 128) * cout * 2:][:ops.bn_partials_numel(m, cout)],
                        zs[lo:lo + n] if sel else None, gam, pkx)
    return run


def split_case(hw, cin, cout):
    x = rnd(B, hw, hw, cin)
    sc, sh = rnd(cin) + 1.5, rnd(cin) * 0.1
    dk, pk = rnd(3, 3, cin, 1), rnd(1, 1, cin, cout) * 0.1
    y = torch.empty(B, hw, hw, cin, device=dev)
    z = torch.empty(B, hw, hw, cout, device=dev)
    part = torch.zeros(ops.bn_partials_numel(B * hw * hw, cout), device=dev)

    def run(lo, n):
        m = n * hw * hw
        ops.dwconv3x3_fwd(View.bnrelu(x[lo:lo + n], sc, sh), n, hw, hw, dk, y[lo:lo + n])
        ops.pointwise_fwd(y[lo:lo + n], m, cin, cout, pk, z[lo:lo + n],
                          part[(lo * hw * hw // 128) * cout * 2:][:ops.bn_partials_numel(m, cout)])
    return run


def convt_case(hw, cin, cout):
    x = rnd(B, hw, hw, cin)
    k, b = rnd(2, 2, cout, cin) * 0.1, rnd(cout)
    out = torch.empty(B, 2 * hw, 2 * hw, cout, device=dev)

    def run(lo, n):
        ops.conv_transpose2x2_fwd(View.plain(x[lo:lo + n]), n, hw, hw, cout, k, b, out[lo:lo + n])
    return run


CASES = [("enc1_block2 fused", sep_case(256, 64, 64, True)), ("enc2_block2 fused", sep_case(128, 128, 128, True)),
         ("enc3_block2 fused", sep_case(64, 256, 256, True)), ("enc4_block2 dw+pw", split_case(32, 512, 512)),
         ("bneck_block2 dw+pw", split_case(16, 1024, 1024)), ("dec2_upsample convT", convt_case(64, 256, 128)),
         ("dec4_upsample convT", convt_case(16, 1024, 512))]


def timed(fn, reps=10):
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[1]


def main():
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    for name, run in CASES:
        full = lambda: run(0, B)

        def halves():
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                run(0, B // 2)
            with torch.cuda.stream(s2):
                run(B // 2, B // 2)
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        def seq_halves():
            run(0, B // 2)
            run(B // 2, B // 2)
        for f in (full, halves, seq_halves):
            f()
        torch.cuda.synchronize()
        r = {"op": name, "us_full": round(timed(full), 1), "us_two_streams": round(timed(halves), 1),
             "us_two_halves_one_stream": round(timed(seq_halves), 1)}
        r["gain"] = round(r["us_full"] / r["us_two_streams"], 3)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
