"""Input pipeline of scripts/train.py (reference :169-220) for the engine: paired image/mask
batches with Keras `flow_from_directory` semantics — sorted file listing, RGB frames resized
bilinear, grayscale masks resized nearest, rescale 1/255 on both, per-sample horizontal flip
shared by image and mask (the reference synchronises the two generators through seed 2301),
shuffling for training only.  Data-parallel: every rank walks the same global batch order and
keeps its own shard of each global batch, so N ranks x (batch/N) == one global batch.

Decoding runs on the host (PIL); batches are handed to the GPU as pinned tensors.  The exact
Keras RNG stream is not reproduced (TF's generator is not portable).
"""
from __future__ import annotations

import os
from typing import Iterator, Tuple

import numpy as np

from .dp import shard_bounds

IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".ppm")


def _list(d):
    if not os.path.isdir(d):
        raise FileNotFoundError(f"directory not found: {d}")
    return sorted(f for f in os.listdir(d) if f.lower().endswith(IMG_EXT))


def load_image(path, size, mode):
    from PIL import Image
    im = Image.open(path).convert("RGB" if mode == "rgb" else "L")
    if im.size != (size[1], size[0]):
        im = im.resize((size[1], size[0]), Image.BILINEAR if mode == "rgb" else Image.NEAREST)
    a = np.asarray(im, dtype=np.float32) / 255.0
    return a if a.ndim == 3 else a[..., None]


class PairLoader:
    def __init__(self, frames_dir, masks_dir, size, batch_size, seed, shuffle=True, horizontal_flip=False, rank=0,
                 world=1):
        self.frames = [os.path.join(frames_dir, f) for f in _list(frames_dir)]
        self.masks = [os.path.join(masks_dir, f) for f in _list(masks_dir)]
        if len(self.frames) != len(self.masks):
            raise ValueError(f"{len(self.frames)} frames but {len(self.masks)} masks")
        self.size, self.batch_size, self.seed = size, batch_size, seed
        self.shuffle, self.flip, self.rank, self.world = shuffle, horizontal_flip, rank, world
        self.samples = len(self.frames)

    def __iter__(self) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
        epoch = 0
        while True:
            rng = np.random.default_rng(self.seed + epoch)
            order = rng.permutation(self.samples) if self.shuffle else np.arange(self.samples)
            flips = rng.random(self.samples) < 0.5 if self.flip else np.zeros(self.samples, bool)
            for b0 in range(0, self.samples, self.batch_size):
                idx = order[b0:b0 + self.batch_size]
                lo, hi = shard_bounds(len(idx), self.world, self.rank)
                idx = idx[lo:hi]
                xs, ys = [], []
                for i in idx:
                    x = load_image(self.frames[i], self.size, "rgb")
                    y = load_image(self.masks[i], self.size, "grayscale")
                    if flips[i]:
                        x, y = x[:, ::-1], y[:, ::-1]
                    xs.append(x)
                    ys.append(y)
                yield np.ascontiguousarray(np.stack(xs)), np.ascontiguousarray(np.stack(ys))
            epoch += 1


class synthetic_pairs:
    """N synthetic (image, mask) pairs: U[0,1) images, ID-card-like quad masks (~30% fg)."""

    def __init__(self, n, size, batch_size, seed, shuffle=True, rank=0, world=1):
        self.samples, self.size, self.batch_size, self.seed = n, size, batch_size, seed
        self.shuffle, self.rank, self.world = shuffle, rank, world

    def _pair(self, i):
        rng = np.random.default_rng(self.seed * 1000003 + i)
        h, w = self.size
        x = rng.random((h, w, 3), dtype=np.float32)
        y = np.zeros((h, w, 1), np.float32)
        hh, ww = int(h * rng.uniform(0.4, 0.7)), int(w * rng.uniform(0.4, 0.7))
        y0, x0 = rng.integers(0, h - hh), rng.integers(0, w - ww)
        y[y0:y0 + hh, x0:x0 + ww] = 1.0
        x[y0:y0 + hh, x0:x0 + ww] = 0.5 * x[y0:y0 + hh, x0:x0 + ww] + 0.5  # a learnable "card"
        return x, y

    def __iter__(self):
        epoch = 0
        while True:
            rng = np.random.default_rng(self.seed + epoch)
            order = rng.permutation(self.samples) if self.shuffle else np.arange(self.samples)
            for b0 in range(0, self.samples, self.batch_size):
                idx = order[b0:b0 + self.batch_size]
                lo, hi = shard_bounds(len(idx), self.world, self.rank)
                pairs = [self._pair(int(i)) for i in idx[lo:hi]]
                yield np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs])
            epoch += 1
