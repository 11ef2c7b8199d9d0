"""Per-launch listing of ONE training step from a rocprofv3 kernel-trace CSV (the complete step
of median wall time: between two AdamW launches), with durations, grid and resource usage, and a
per-kernel-family total.  usage: python tools/step_trace.py trace.csv [min_us]"""
import csv, re, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
# the step of median wall time among the complete steps (the last one can carry host gaps)
walls = sorted((int(rows[j]["End_Timestamp"]) - int(rows[i + 1]["Start_Timestamp"]), i, j) for i, j in zip(ad, ad[1:]))
_, i0, j0 = walls[len(walls) // 2]
a, b = i0 + 1, j0 + 1
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
tend = int(step[-1]["End_Timestamp"])
fam = defaultdict(float)
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
busy = 0.0
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy += d
    name = r["Kernel_Name"]
    short = re.sub(r"unet::\(anonymous namespace\)::", "", name)
    short = re.sub(r"\(.*$", "", short.replace("void ", ""))
    fam[short] += d
    if d >= mn:
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f}us q{r['Queue_Id']} grid={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']} "
              f"v{r['VGPR_Count']}/a{r['Accum_VGPR_Count']} lds{r['LDS_Block_Size']} {short[:90]}")
print(f"step wall {(tend - t0) / 1e3:.1f} us, kernel busy {busy:.1f} us, launches {len(step)}")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:30]:
    print(f"{v:9.1f}us {k[:110]}")
