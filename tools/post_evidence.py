"""Copy / summarise a tools/gpu_final3.sh session (gpurun_out/) into profiles/ under TAG:
kernel-trace stats (two-stream, single-stream), the median step's launch trace, the bench line,
the parity log, PMC HBM traffic of the roofline op, and enc2_block1's PMC summary.

    python tools/post_evidence.py TAG
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def one(pattern):
    fs = sorted(glob.glob(os.path.join(G, pattern), recursive=True), key=os.path.getmtime)
    return fs[-1] if fs else None


def main():
    tag = sys.argv[1]
    for src, dst in ((f"prof/**/{tag}_kernel_stats.csv", f"{tag}_kernel_stats.csv"),
                     (f"prof/**/{tag}_1s_kernel_stats.csv", f"{tag}_1s_kernel_stats.csv"),
                     (f"parity_{tag}.jsonl", f"{tag}_parity.jsonl")):
        f = one(src)
        if f:
            shutil.copy(f, os.path.join(P, dst))
    lines = [ln for ln in open(os.path.join(G, "bench.log")) if ln.startswith("{")]
    open(os.path.join(P, f"{tag}_bench.log"), "w").write("".join(lines))
    tr = one(f"prof/**/{tag}_kernel_trace.csv")
    if tr:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_trace.py"), tr], capture_output=True,
                             text=True).stdout
        open(os.path.join(P, f"{tag}_step_trace.txt"), "w").write(out)
    fe, wr = one(f"pmc/**/{tag}_fetch_counter_collection.csv"), one(f"pmc/**/{tag}_write_counter_collection.csv")
    if fe and wr:  # the bench line's roofline op (the largest share of the single-stream breakdown), and the GEMM
        ops_ = [json.loads(lines[0])["roofline"]["kernel"], "unet_pointwise_bwd_data_bnrelu_x3"]
        for op in dict.fromkeys(ops_):
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), fe, wr,
                                os.path.join(P, f"{tag}_traffic_{op[5:]}.json"), op], capture_output=True, text=True)
            print(op, r.stdout.strip()[:200], r.stderr.strip()[-200:])
    if fe and wr:  # whole-step HBM bytes (every dispatch of the PMC passes' timed steps)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_step_bytes.py"), fe, wr,
                            os.path.join(G, "bench.log"), os.path.join(P, f"{tag}_step_traffic.json")],
                           capture_output=True, text=True)
        print("step traffic", r.stdout.strip()[:200], r.stderr.strip()[-300:])
    # enc2_block1 forward at batch 32: bytes and the SQ stall group, averaged over its dispatches
    rec = {}
    for kind in ("fetch", "write", "sq"):
        f = one(f"pmc/**/{tag}_e2b1_{kind}_counter_collection.csv")
        if not f:
            continue
        acc = {}
        for r in csv.DictReader(open(f)):
            if "sepconv" not in r["Kernel_Name"]:
                continue
            d = acc.setdefault(r["Dispatch_Id"], {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
        ds = list(acc.values())[2:]  # (first launches warm the caches)
        for k in ds[0]:
            rec[k] = sum(d[k] for d in ds) / len(ds)
    if rec:
        if "FETCH_SIZE" in rec:
            rec["hbm_read_bytes"] = rec["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in rec:
            rec["hbm_write_bytes"] = rec["WRITE_SIZE"] * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in rec:
            rec["mfma_busy_frac"] = rec["SQ_VALU_MFMA_BUSY_CYCLES"] / (rec["dur_ns"] * 2.4 * 1024)
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                rec[k + "_frac"] = rec[k] / rec["SQ_WAVE_CYCLES"]
        rec["what"] = ("enc2_block1 training forward at batch 32 (BN+ReLU view of the pooled selection, 64 -> 128, "
                       "y stored, split-precision MFMA): tools/sep_one.py 1 128 128 64 128 10 x3, N=32; FETCH_SIZE x1024 x2, "
                       "WRITE_SIZE x1024 (gfx950 corrections); per-dispatch averages")
        json.dump(rec, open(os.path.join(P, f"{tag}_pmc_enc2_block1.json"), "w"), indent=1)
    print("ok", tag)


if __name__ == "__main__":
    main()
