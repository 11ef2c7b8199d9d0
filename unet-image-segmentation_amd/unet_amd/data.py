"""Input pipeline of scripts/train.py (reference :169-220) for the engine: paired image/mask
batches with Keras `flow_from_directory` semantics — sorted file listing, RGB frames resized
bilinear, grayscale masks resized nearest, rescale 1/255 on both, per-sample horizontal flip
shared by image and mask (the reference synchronises the two generators through seed 2301),
shuffling for training only.  Data-parallel: every rank walks the same global batch order and
keeps its own shard of each global batch, so N ranks x (batch/N) == one global batch.

Decoding runs on the host (PIL) in a background thread pool, a few batches ahead of the step
(`Prefetcher`), and each batch is copied into page-locked host memory and sent to the device
with a non-blocking copy on a dedicated stream, so neither decoding nor the H2D copy sits on the
train step's critical path.  The exact Keras RNG stream is not reproduced (TF's generator is
not portable).

Data-parallel sharding: with W ranks every global batch of B samples is cut into W shards
(remainder to the low ranks; `dp.shard_bounds`).  A trailing global batch with fewer than W
samples would leave some rank without a sample, so it is skipped on every rank alike.  Each
yielded batch carries `global_size` (the samples of the whole global batch), from which the
engine weights its shard's loss gradient (model.train_step).
"""
from __future__ import annotations

import os
import threading
from typing import Iterator, Tuple

import numpy as np

from .dp import shard_bounds


def default_cache_cap() -> int:
    """A quarter of the host's physical memory (the node-wide budget of the default decode caches)."""
    try:
        return os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE") // 4
    except (ValueError, OSError, AttributeError):
        return 64 << 30


def local_world_size() -> int:
    """Data-parallel ranks on this host (torchrun's LOCAL_WORLD_SIZE; 1 without a launcher)."""
    try:
        return max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    except ValueError:
        return 1


class Shard(tuple):
    """(images, masks) of this rank's shard; .global_size = samples in the whole global batch."""

    global_size: int = 0

    def __new__(cls, x, y, global_size):
        t = super().__new__(cls, (x, y))
        t.global_size = int(global_size)
        return t


def global_batches(samples: int, batch_size: int, world: int):
    """[start, stop) of the global batches of one pass over `samples` (trailing batches with
    fewer samples than ranks are dropped: every rank must get at least one)."""
    for b0 in range(0, samples, batch_size):
        b1 = min(b0 + batch_size, samples)
        if b1 - b0 >= world:
            yield b0, b1

IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".ppm")


def _list(d):
    if not os.path.isdir(d):
        raise FileNotFoundError(f"directory not found: {d}")
    return sorted(f for f in os.listdir(d) if f.lower().endswith(IMG_EXT))


def load_image_u8(path, size, mode):
    """Decoded + resized image as uint8 HWC (bilinear for RGB frames, nearest for masks)."""
    from PIL import Image
    im = Image.open(path).convert("RGB" if mode == "rgb" else "L")
    if im.size != (size[1], size[0]):
        im = im.resize((size[1], size[0]), Image.BILINEAR if mode == "rgb" else Image.NEAREST)
    a = np.asarray(im, dtype=np.uint8)
    return a if a.ndim == 3 else a[..., None]


def load_image(path, size, mode):
    return load_image_u8(path, size, mode).astype(np.float32) / 255.0


class PairLoader:
    """cache_bytes: decoded, resized samples are kept as uint8 (256 x 256 x 4 B = 256 KiB per
    pair at 256 x 256) up to this budget, so PNG decoding (~25 ms per 960 x 540 frame on one core,
    tools/bench_loader.py) is paid once per file, not once per epoch: the decode and resize are
    deterministic, so the batches are identical to decoding every epoch.  Default: 16 GiB per
    loader (about 64k pairs at 256 x 256, whatever the rank count); a host-wide budget for all of
    a node's loaders can be set with UNET_LOADER_CACHE_HOST_GB (divided among the node's ranks and
    their train + val loaders).  No loader throughput was measured at 8 ranks, so the default does
    not shrink with the rank count."""

    def __init__(self, frames_dir, masks_dir, size, batch_size, seed, shuffle=True, horizontal_flip=False, rank=0,
                 world=1, workers=16, cache_bytes=None):
        if batch_size < world:
            raise ValueError(f"batch size {batch_size} < {world} data-parallel ranks: every rank needs a sample")
        self.frames = [os.path.join(frames_dir, f) for f in _list(frames_dir)]
        self.masks = [os.path.join(masks_dir, f) for f in _list(masks_dir)]
        if len(self.frames) != len(self.masks):
            raise ValueError(f"{len(self.frames)} frames but {len(self.masks)} masks")
        self.size, self.batch_size, self.seed = size, batch_size, seed
        self.shuffle, self.flip, self.rank, self.world = shuffle, horizontal_flip, rank, world
        self.samples = len(self.frames)
        self.workers = max(1, int(workers))
        self._pool = None
        if cache_bytes is None:
            host_gb = os.environ.get("UNET_LOADER_CACHE_HOST_GB")
            if host_gb:  # one host-wide budget over this node's ranks x (train + val) loaders
                cache_bytes = int(float(host_gb) * (1 << 30)) // (2 * local_world_size())
            else:  # 16 GiB per loader, clamped so this node's ranks x (train + val) loaders stay
                # within a quarter of physical memory (8 ranks x 2 loaders x 16 GiB)
                cache_bytes = min(16 << 30, default_cache_cap() // (2 * local_world_size()))
        self.cache_bytes = int(cache_bytes)
        self._cache = {}
        self._cached_bytes = 0
        self._lock = threading.Lock()

    def __iter__(self) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
        epoch = 0
        while True:
            rng = np.random.default_rng(self.seed + epoch)
            order = rng.permutation(self.samples) if self.shuffle else np.arange(self.samples)
            flips = rng.random(self.samples) < 0.5 if self.flip else np.zeros(self.samples, bool)
            for b0, b1 in global_batches(self.samples, self.batch_size, self.world):
                idx = order[b0:b1]
                lo, hi = shard_bounds(len(idx), self.world, self.rank)
                yield Shard(*self.load(idx[lo:hi], flips), global_size=len(idx))
            epoch += 1

    def _sample(self, i, flip):
        xy = self._cache.get(i)
        if xy is None:
            xy = (load_image_u8(self.frames[i], self.size, "rgb"), load_image_u8(self.masks[i], self.size, "grayscale"))
            nb = xy[0].nbytes + xy[1].nbytes
            with self._lock:  # decode threads share the budget: check-and-add as one step
                if i not in self._cache and self._cached_bytes + nb <= self.cache_bytes:
                    self._cache[i] = xy
                    self._cached_bytes += nb
        x = xy[0].astype(np.float32) / 255.0  # rescale=1/255 (reference scripts/train.py:170-178)
        y = xy[1].astype(np.float32) / 255.0
        if flip:
            x, y = x[:, ::-1], y[:, ::-1]
        return x, y

    def load(self, idx, flips):
        """Decode the samples idx (PIL releases the GIL while decoding / resizing, so a small
        thread pool decodes a batch in parallel); returns contiguous (x, y) batches."""
        if self.workers > 1 and len(idx) > 1:
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._pool = ThreadPoolExecutor(self.workers, thread_name_prefix="unet-decode")
            pairs = list(self._pool.map(lambda i: self._sample(int(i), bool(flips[i])), idx))
        else:
            pairs = [self._sample(int(i), bool(flips[i])) for i in idx]
        return (np.ascontiguousarray(np.stack([p[0] for p in pairs])),
                np.ascontiguousarray(np.stack([p[1] for p in pairs])))


class synthetic_pairs:
    """N synthetic (image, mask) pairs: U[0,1) images, ID-card-like quad masks (~30% fg)."""

    def __init__(self, n, size, batch_size, seed, shuffle=True, rank=0, world=1):
        if batch_size < world:
            raise ValueError(f"batch size {batch_size} < {world} data-parallel ranks: every rank needs a sample")
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
            for b0, b1 in global_batches(self.samples, self.batch_size, self.world):
                idx = order[b0:b1]
                lo, hi = shard_bounds(len(idx), self.world, self.rank)
                pairs = [self._pair(int(i)) for i in idx[lo:hi]]
                yield Shard(np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs]), global_size=len(idx))
            epoch += 1
