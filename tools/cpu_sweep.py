"""CPU-baseline thread sweep: the TF-CPU proxy train step (bench.cpu_baseline)
at several thread counts on this host, one JSON line each.

    python tools/cpu_sweep.py OUT.jsonl [threads ...]   (default 16 64 128)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]

import bench  # noqa: E402


def main():
    out = sys.argv[1]
    threads = [int(t) for t in sys.argv[2:]] or [16, 64, 128]
    for t in threads:
        r = bench.cpu_baseline(256, 1, 16, warmup=2, steps=3, threads=t)
        r["threads_requested"] = t
        print(json.dumps(r), flush=True)
        with open(out, "a") as f:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
