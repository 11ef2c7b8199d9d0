"""Host-side input pipeline (scripts/train.py:169-220 restated in unet_amd/data.py) and the
background prefetcher (unet_amd/prefetch.py), on CPU."""
import os
import threading

import numpy as np
import pytest
from PIL import Image

from unet_amd.data import PairLoader, Shard, global_batches, load_image, synthetic_pairs
from unet_amd.dp import shard_bounds
from unet_amd.prefetch import Prefetcher


def _write_dataset(root, n, size=(40, 30)):
    fr, mk = os.path.join(root, "frames"), os.path.join(root, "masks")
    os.makedirs(fr)
    os.makedirs(mk)
    rng = np.random.default_rng(0)
    for i in range(n):
        Image.fromarray(rng.integers(0, 256, (size[1], size[0], 3), dtype=np.uint8)).save(
            os.path.join(fr, f"f{i:03d}.png"))
        m = np.zeros((size[1], size[0]), np.uint8)
        m[5:5 + i % 7 + 3, 4:20] = 255
        Image.fromarray(m).save(os.path.join(mk, f"f{i:03d}.png"))
    return fr, mk


def test_global_batches_drop_only_unshardable_tail():
    assert list(global_batches(10, 4, 1)) == [(0, 4), (4, 8), (8, 10)]
    assert list(global_batches(10, 4, 2)) == [(0, 4), (4, 8), (8, 10)]
    assert list(global_batches(9, 4, 2)) == [(0, 4), (4, 8)]          # 1 sample left < 2 ranks
    assert list(global_batches(11, 4, 4)) == [(0, 4), (4, 8)]
    assert list(global_batches(5, 5, 2)) == [(0, 5)]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_pair_loader_shards_cover_each_global_batch(tmp_path, world):
    fr, mk = _write_dataset(str(tmp_path), 7)
    seen = {}
    for rank in range(world):
        ld = PairLoader(fr, mk, (16, 16), 3, seed=2301, shuffle=True, horizontal_flip=True, rank=rank, world=world,
                        workers=2)
        it = iter(ld)
        nb = len(list(global_batches(7, 3, world)))
        for b in range(nb):
            s = next(it)
            assert isinstance(s, Shard) and s.global_size in (3, 1)
            x, y = s
            assert x.shape[1:] == (16, 16, 3) and y.shape[1:] == (16, 16, 1)
            assert x.dtype == np.float32 and 0 <= x.min() and x.max() <= 1
            lo, hi = shard_bounds(s.global_size, world, rank)
            assert x.shape[0] == hi - lo >= 1
            seen.setdefault(b, []).append(x)
    for b, parts in seen.items():  # the shards of every rank tile the global batch
        assert sum(p.shape[0] for p in parts) in (3, 1)


def test_pair_loader_decode_threads_match_serial(tmp_path):
    fr, mk = _write_dataset(str(tmp_path), 6)
    a = next(iter(PairLoader(fr, mk, (16, 16), 6, seed=1, workers=4)))
    b = next(iter(PairLoader(fr, mk, (16, 16), 6, seed=1, workers=1)))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_pair_loader_rejects_batch_below_world(tmp_path):
    fr, mk = _write_dataset(str(tmp_path), 4)
    with pytest.raises(ValueError):
        PairLoader(fr, mk, (16, 16), 1, seed=1, world=2)
    with pytest.raises(ValueError):
        synthetic_pairs(8, (16, 16), 1, 1, world=2)


def test_load_image_rescale_and_modes(tmp_path):
    p = os.path.join(str(tmp_path), "m.png")
    Image.fromarray(np.full((8, 8), 255, np.uint8)).save(p)
    m = load_image(p, (4, 4), "grayscale")
    assert m.shape == (4, 4, 1) and np.all(m == 1.0)


def test_synthetic_pairs_remainder_batch_sharded():
    sp = synthetic_pairs(5, (16, 16), 5, seed=3, shuffle=False, rank=1, world=2)
    s = next(iter(sp))
    assert s.global_size == 5 and s[0].shape[0] == 2  # ranks get 3 and 2


def test_prefetcher_cpu_order_and_global_size():
    src = synthetic_pairs(9, (8, 8), 3, seed=3, shuffle=False)
    ref = [next(iter(src)) for _ in range(1)]
    pf = Prefetcher(src, device="cpu", depth=2)
    it = iter(pf)
    got = [next(it) for _ in range(3)]
    pf.close()
    assert np.array_equal(got[0][0].numpy(), ref[0][0])
    assert all(g.global_size == 3 for g in got)


def test_prefetcher_propagates_errors_and_stops():
    def bad():
        yield np.zeros((1, 2, 2, 3)), np.zeros((1, 2, 2, 1))
        raise RuntimeError("decode failed")
    it = iter(Prefetcher(bad(), device="cpu"))
    next(it)
    with pytest.raises(RuntimeError, match="decode failed"):
        next(it)
    n0 = threading.active_count()
    pf = Prefetcher(synthetic_pairs(100, (8, 8), 2, seed=1), device="cpu", depth=2)
    it = iter(pf)
    next(it)
    pf.close()
    assert threading.active_count() <= n0 + 1


def test_prefetcher_finite_source_ends():
    items = [(np.ones((1, 2, 2, 3)) * i, np.zeros((1, 2, 2, 1))) for i in range(4)]
    out = list(Prefetcher(items, device="cpu", depth=1))
    assert [float(o[0][0, 0, 0, 0]) for o in out] == [0, 1, 2, 3]


def test_prefetcher_limit_keeps_single_pass_generator_batches():
    """A shared one-shot generator loses no batches to read-ahead (evaluate on a
    Keras-style flow): with limit=k the producer pulls exactly k batches per iteration."""
    def gen():
        i = 0
        while True:
            yield np.full((1, 2, 2, 3), i, np.float32), np.zeros((1, 2, 2, 1), np.float32)
            i += 1
    g = gen()
    for epoch in range(3):
        it = iter(Prefetcher(g, device="cpu", depth=4, limit=2))
        got = [float(next(it)[0][0, 0, 0, 0]) for _ in range(2)]
        assert got == [2 * epoch, 2 * epoch + 1]
        with pytest.raises(StopIteration):
            next(it)


def test_prefetcher_restart_isolates_iterations():
    """Re-iterating one Prefetcher: the previous producer is joined before a new one starts, so a
    late producer can never push batches of the old iteration into the new queue."""
    import time

    class Slow:
        def __iter__(self):
            i = 0
            while True:
                time.sleep(0.01)
                yield np.full((1, 2, 2, 3), i, np.float32), np.zeros((1, 2, 2, 1), np.float32)
                i += 1
    pf = Prefetcher(Slow(), device="cpu", depth=2)
    for _ in range(4):
        it = iter(pf)
        first = [float(next(it)[0][0, 0, 0, 0]) for _ in range(3)]
        assert first == [0.0, 1.0, 2.0]  # every iteration starts a fresh pass of the source
    pf.close()
    assert pf._thread is None
