"""Input prefetch off the step's critical path (the reference's ImageDataGenerator pipeline,
scripts/train.py:169-220, runs synchronously in the step loop; here it runs beside it).

A background thread pulls host batches from a loader (PairLoader decodes its samples with a
thread pool), copies each batch into page-locked memory and issues a non-blocking H2D copy on
its own HIP stream; the consumer's stream waits on an event recorded after the copy, so the
step never blocks on decoding or on PCIe unless the loader falls behind.  `depth` batches are
kept in flight (bounded queue).  Errors raised by the loader are re-raised in the consumer.
"""
from __future__ import annotations

import queue
import threading
from typing import Iterable, Optional

import numpy as np
import torch

_END = object()


class _Failure:
    def __init__(self, exc: BaseException):
        self.exc = exc


class Prefetcher:
    """Iterates `source` (yielding (x, y) numpy batches, optionally with .global_size) and yields
    (x, y) device tensors (a `data.Shard` when the source batch carries global_size)."""

    def __init__(self, source: Iterable, device=None, depth: int = 3):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.source = source
        self.device = torch.device(device) if device is not None else None
        self.depth = depth
        self._q: Optional[queue.Queue] = None
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()

    # ------------------------------------------------------------------ producer ---
    def _to_device(self, arr, stream):
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32))
        if self.device is None or self.device.type != "cuda":
            return t, None
        pinned = t.pin_memory()
        with torch.cuda.stream(stream):
            d = pinned.to(self.device, non_blocking=True)
        return d, pinned

    def _run(self):
        stream = None
        try:
            if self.device is not None and self.device.type == "cuda":
                torch.cuda.set_device(self.device)
                stream = torch.cuda.Stream(device=self.device)
            for batch in self.source:
                if self._stop.is_set():
                    break
                x, y = batch[0], batch[1]
                gsz = getattr(batch, "global_size", None)
                xd, xp = self._to_device(x, stream)
                yd, yp = self._to_device(y, stream)
                ev = None
                if stream is not None:
                    ev = torch.cuda.Event()
                    ev.record(stream)
                item = (xd, yd, gsz, ev, (xp, yp))  # pinned buffers stay referenced until consumed
                while not self._stop.is_set():
                    try:
                        self._q.put(item, timeout=0.1)
                        break
                    except queue.Full:
                        continue
            self._put_final(_END)
        except BaseException as e:  # surfaced in the consumer
            self._put_final(_Failure(e))

    def _put_final(self, item):
        while not self._stop.is_set():
            try:
                self._q.put(item, timeout=0.1)
                return
            except queue.Full:
                continue

    # ------------------------------------------------------------------ consumer ---
    def __iter__(self):
        self.close()
        self._stop.clear()
        self._q = queue.Queue(maxsize=self.depth)
        self._thread = threading.Thread(target=self._run, name="unet-prefetch", daemon=True)
        self._thread.start()
        return self

    def __next__(self):
        if self._q is None:
            iter(self)
        item = self._q.get()
        if item is _END:
            self.close()
            raise StopIteration
        if isinstance(item, _Failure):
            self.close()
            raise item.exc
        xd, yd, gsz, ev, _pinned = item
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            xd.record_stream(cur)
            yd.record_stream(cur)
        if gsz is not None:
            from .data import Shard
            return Shard(xd, yd, gsz)
        return xd, yd

    def close(self):
        self._stop.set()
        t = self._thread
        if t is not None and t.is_alive():
            t.join(timeout=5.0)
        self._thread = None
        self._q = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
