"""HBM traffic per launch of the roofline op from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE, separate runs of the same bench command, kernel-trace only).

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts half the bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores.  Infinity-Cache hits are counted as fetches, so this is an
upper bound on HBM bytes.  The summary records the sha256 (first 16 hex digits) of the library
build it measured (`lib_sha16`); bench.py only quotes a summary whose hash matches the library
it runs.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [OP]
"""
import csv
import hashlib
import json
import os
import re
import sys

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "unet-image-segmentation_amd",
                   "unet_amd", "libunet_hip.so")


def lib_sha16(path=LIB):
    """sha256 of the library build, first 16 hex digits (None if it is not built)."""
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None

# the kernels each C-ABI op launches (training-mode epilogues); the optional trailing flag is the
# split-precision (X6) template parameter, false in the product library
OPS = {
    "unet_pointwise_fwd": r"gemm_rows_vec<\d+, \d+, \d+, 0, false, 1(, (true|false))?>|gemm_rows_kernel<\d+, \d+, 0, false, 1>",
    "unet_pointwise_bwd_data": r"gemm_rows_vec<\d+, \d+, \d+, 0, false, 0(, (true|false))?>|gemm_rows_kernel<\d+, \d+, 0, false, 0>",
    "unet_pointwise_bwd_filter": r"gemm_wgrad_(vec|kernel)<\d+, \d+, 0, false, 0, false(, (true|false))?>",
    "unet_sepconv_fwd": r"sepconv_(fwd|rk|px)_kernel<",
    "unet_sepconv_bwd_filter": r"sepconv_wgrad_kernel<",
    "unet_pointwise_bwd_data_bnrelu": r"gemm_rows_vec<\d+, \d+, \d+, 3, (true|false), 0, (true|false)(, (true|false))?>",
    # (round 6: the split-precision route's launches -- X6 = true -- and the fp32 fall-backs of the same op)
    "unet_pointwise_bwd_data_bnrelu_x3": r"gemm_rows_vec<\d+, \d+, \d+, 3, (true|false), 0, (true|false)(, (true|false))?>",
    "unet_conv_transpose2x2_bwd_data_bnstats": r"gemm_rows_vec<\d+, \d+, \d+, 2, false, 3, (true|false)(, (true|false))?>",
    "unet_pointwise_bwd_data_bnrelu_wgrad": r"img_pw_bwd_kernel<",
}


def per_launch(path, pat):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if re.search(pat, r["Kernel_Name"])]
    return len(vals), (sum(vals) / len(vals) * 1024.0 if vals else None)


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    op = sys.argv[4] if len(sys.argv) > 4 else "unet_pointwise_fwd"
    pat = OPS[op]
    nf, f = per_launch(fetch_csv, pat)
    nw, w = per_launch(write_csv, pat)
    if f is None or w is None:
        raise SystemExit(f"no dispatches of {op} in the counter files")
    res = {"op": op, "kernel_regex": pat, "dispatches": [nf, nw],
           "fetch_bytes_per_launch_raw": round(f), "fetch_bytes_per_launch": round(2 * f),
           "write_bytes_per_launch": round(w), "traffic_bytes_per_launch": round(2 * f + w),
           "sources": [fetch_csv, write_csv], "lib_sha16": lib_sha16(),
           "correction": "FETCH_SIZE x1024 x2 (gfx950 half-count of wide reads), WRITE_SIZE x1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
