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

    def __init__(self, source: Iterable, device=None, depth: int = 3, limit: Optional[int] = None):
        """limit: pull at most this many batches from `source` per iteration, so a single-pass
        generator shared with the caller loses no batches to read-ahead (model.fit / evaluate
        pass the number of steps they will take)."""
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.source = source
        self.limit = limit
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

    def _run(self, q: "queue.Queue", stop: threading.Event):
        """Producer of ONE iteration: it only ever touches its own queue and stop event, so a
        thread that outlives its iteration cannot feed a later one."""
        stream = None
        try:
            if self.device is not None and self.device.type == "cuda":
                torch.cuda.set_device(self.device)
                stream = torch.cuda.Stream(device=self.device)
            taken = 0
            for batch in self.source:
                if stop.is_set():
                    break
                taken += 1
                x, y = batch[0], batch[1]
                gsz = getattr(batch, "global_size", None)
                xd, xp = self._to_device(x, stream)
                yd, yp = self._to_device(y, stream)
                ev = None
                if stream is not None:
                    ev = torch.cuda.Event()
                    ev.record(stream)
                item = (xd, yd, gsz, ev, (xp, yp))  # pinned buffers stay referenced until consumed
                if not self._put(q, stop, item):
                    break
                if self.limit is not None and taken >= self.limit:
                    break
            self._put(q, stop, _END)
        except BaseException as e:  # surfaced in the consumer
            self._put(q, stop, _Failure(e))

    @staticmethod
    def _put(q, stop, item) -> bool:
        while not stop.is_set():
            try:
                q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    # ------------------------------------------------------------------ consumer ---
    def __iter__(self):
        self.close()
        self._stop = threading.Event()  # per iteration: see _run
        self._q = queue.Queue(maxsize=self.depth)
        self._thread = threading.Thread(target=self._run, args=(self._q, self._stop), name="unet-prefetch",
                                        daemon=True)
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

    def close(self, timeout: float = 60.0):
        """Stop the producer and wait for it.  It notices the stop flag between batches, so this
        waits at most for the batch the source is producing; a producer still alive after
        `timeout` (a source blocked inside next()) raises rather than letting a new iteration call
        into the same source concurrently."""
        self._stop.set()
        t = self._thread
        if t is not None and t.is_alive() and t is not threading.current_thread():
            t.join(timeout=timeout)
            if t.is_alive():
                raise RuntimeError("Prefetcher: the producer thread did not stop (source blocked in next())")
        self._thread = None
        self._q = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
