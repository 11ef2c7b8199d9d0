"""Input-pipeline throughput: PairLoader decoding a
MIDV-layout dataset of 960x540 PNG frames + masks (the half-resolution frames
scripts/download_dataset_midv.py writes, reference :69-70,136-139) and resizing them to 256x256
(bilinear frames, nearest masks, /255), at several decode-thread counts, in images/s -- to set
against the device train step's rate at configs[1].

    python tools/bench_loader.py OUT.jsonl [workers ...]     (default 4 8 16)

The frames are the reference's two sample photos (tests/golden/samples) under per-file crops,
flips and brightness changes, so they compress and decode like camera frames; masks are quads.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]

SAMPLES = os.path.join(ROOT, "tests", "golden", "samples")
SPLITS = ("train", "val")


def make_midv_tree(root, n_train, n_val, seed=2301, size=(960, 540)):
    """dataset/train/{train,val}_{frames,masks}/image/imageK.png under `root` (the layout of
    reference scripts/train.py:77-90): RGB frames from the sample photos, binary quad masks."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    photos = [np.asarray(Image.open(os.path.join(SAMPLES, f)).convert("RGB"))
              for f in sorted(os.listdir(SAMPLES)) if f.endswith(".png")]
    w, h = size
    for split, n in zip(SPLITS, (n_train, n_val)):
        fd = os.path.join(root, "dataset", "train", f"{split}_frames", "image")
        md = os.path.join(root, "dataset", "train", f"{split}_masks", "image")
        os.makedirs(fd, exist_ok=True)
        os.makedirs(md, exist_ok=True)
        for i in range(n):
            ph = photos[i % len(photos)]
            im = Image.fromarray(ph).resize((w, h), Image.BILINEAR)
            a = np.asarray(im).astype(np.float32) * rng.uniform(0.7, 1.2)
            if rng.random() < 0.5:
                a = a[:, ::-1]
            Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(os.path.join(fd, f"image{i}.png"))
            m = np.zeros((h, w), np.uint8)
            hh, ww = int(h * rng.uniform(0.4, 0.7)), int(w * rng.uniform(0.4, 0.7))
            y0, x0 = rng.integers(0, h - hh), rng.integers(0, w - ww)
            m[y0:y0 + hh, x0:x0 + ww] = 255
            Image.fromarray(m).save(os.path.join(md, f"image{i}.png"))
    return os.path.join(root, "dataset", "train")


def main():
    from unet_amd.data import PairLoader
    out = sys.argv[1] if len(sys.argv) > 1 else None
    workers = [int(w) for w in sys.argv[2:]] or [4, 8, 16]
    batch, n_batches = 16, 8
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        base = make_midv_tree(d, batch * n_batches, batch)
        print(f"dataset written in {time.perf_counter() - t0:.1f} s", flush=True)
        for wk in workers:
            ld = PairLoader(os.path.join(base, "train_frames", "image"), os.path.join(base, "train_masks", "image"),
                            (256, 256), batch, 2301, shuffle=True, horizontal_flip=True, workers=wk)
            it = iter(ld)
            rates = []
            for _ in range(2):  # epoch 1 decodes every file; epoch 2 reads the decoded cache
                t = time.perf_counter()
                for _ in range(n_batches):
                    x, y = next(it)
                rates.append(batch * n_batches / (time.perf_counter() - t))
            assert x.shape == (batch, 256, 256, 3) and y.shape == (batch, 256, 256, 1)
            r = {"workers": wk, "first_epoch_images_per_s": round(rates[0], 1),
                 "cached_epoch_images_per_s": round(rates[1], 1), "batches_per_epoch": n_batches,
                 "batch": batch, "frame": "960x540 PNG -> 256x256", "cpus": len(os.sched_getaffinity(0))}
            print(json.dumps(r), flush=True)
            if out:
                with open(out, "a") as f:
                    f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
