"""Whole-step HBM traffic from a bench run's rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(tools/gpu_final3.sh: 1 warm-up + 3 timed steps, single PMC pass each): bytes per step summed over
every dispatch of the timed steps, per kernel family, and the average bandwidth against the step
time of the same tree's bench line.  FETCH_SIZE x 1024 x 2, WRITE_SIZE x 1024 (the guide's gfx950
corrections; Infinity-Cache hits count as fetches, so reads are an upper bound).

    python tools/pmc_step_bytes.py FETCH.csv WRITE.csv BENCH.log OUT.json
"""
import collections
import csv
import json
import sys


def per_dispatch(path, mult):
    disp, names = collections.defaultdict(float), {}
    for r in csv.DictReader(open(path)):
        disp[int(r["Dispatch_Id"])] += float(r["Counter_Value"]) * mult
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return disp, names


def main():
    fe, wr, bench, out = sys.argv[1:5]
    res = {}
    fam = collections.defaultdict(lambda: [0.0, 0.0])
    for kind, path, mult in (("read", fe, 2048), ("write", wr, 1024)):
        disp, names = per_dispatch(path, mult)
        ids = sorted(disp)
        # step boundaries: the AdamW launch ends every train step; keep the last 3 steps
        ends = [i for i in ids if "adamw" in names[i]]
        first = ends[-4] if len(ends) >= 4 else ids[0] - 1
        sel = [i for i in ids if first < i <= ends[-1]]
        nsteps = min(3, len(ends))
        res[kind + "_bytes_per_step"] = sum(disp[i] for i in sel) / nsteps
        for i in sel:
            k = names[i].replace("(anonymous namespace)", "").replace("void ", "").split("(")[0]
            k = k.split("<")[0].split("::")[-1] + ("<" + k.split("<", 1)[1][:24] if "<" in k else "")
            fam[k][0 if kind == "read" else 1] += disp[i] / nsteps
    line = next(json.loads(l) for l in open(bench) if l.startswith("{"))
    ms = line["ms_per_step"]
    tot = res["read_bytes_per_step"] + res["write_bytes_per_step"]
    res.update({"ms_per_step": ms, "bytes_per_step": tot, "avg_TBps": tot / (ms * 1e-3) / 1e12,
                "families": {k: {"read_MB": round(v[0] / 1e6, 1), "write_MB": round(v[1] / 1e6, 1)}
                             for k, v in sorted(fam.items(), key=lambda x: -(x[1][0] + x[1][1]))}})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("bytes_per_step", "avg_TBps", "ms_per_step")}))


if __name__ == "__main__":
    main()
