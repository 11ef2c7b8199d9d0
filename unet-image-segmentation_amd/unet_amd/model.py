"""Keras-Model-like facade over UNetEngine: what `U_NET(...)` returns.

Mirrors the parts of tf.keras.Model the reference uses: compile (scripts/train.py:227-234),
fit (:308-316), predict (scripts/inference.py:116, benchmark.py:254), summary (:235),
weights by Keras names, save / load of the trained weights.
"""
from __future__ import annotations

import math
import time
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L
from .dp import GradBucketer
from .engine import UNetEngine
from .metrics import MeanIoU, as_device_tensor
from .optim import AdamW
from .params import FILTERS


def _loss_kind(loss) -> int:
    name = loss if isinstance(loss, str) else getattr(loss, "__name__", "")
    if name in ("dice_loss", "dice"):
        return L.LOSS_DICE
    if name in ("iou_loss", "jaccard_loss", "iou"):
        return L.LOSS_IOU
    raise ValueError(f"unsupported loss {loss!r}: the engine implements dice_loss and iou_loss/jaccard_loss")


class History:
    def __init__(self):
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []


class UNetModel:
    def __init__(self, input_size, num_classes: int = 1, dropout_rate: float = 0.2, use_batch_norm: bool = True,
                 filters: Sequence[int] = FILTERS, device=None, seed: int = 2301, name: str = "U-NET-Segmentation"):
        self.engine = UNetEngine(input_size, num_classes, dropout_rate, use_batch_norm, filters, device, seed)
        self.name = name
        self.input_shape = (None, self.engine.h, self.engine.w, self.engine.c)
        self.output_shape = (None, self.engine.h, self.engine.w, num_classes)
        self.optimizer: Optional[AdamW] = None
        self.loss_kind = L.LOSS_DICE
        self.metric_names: List[str] = []
        self.mean_iou: Optional[MeanIoU] = None
        self.bucketer: Optional[GradBucketer] = None
        # bench.py: a list collecting (end of backward, all-reduce done) HIP event pairs per step
        self.dp_probe: Optional[list] = None
        self.stop_training = False

    # --------------------------------------------------------------------- keras API ---
    @property
    def num_classes(self):
        return self.engine.num_classes

    def compile(self, optimizer=None, loss="dice_loss", metrics: Optional[Iterable] = None):
        self.optimizer = optimizer if optimizer is not None else AdamW()
        self.loss_kind = _loss_kind(loss)
        self.metric_names = []
        self.mean_iou = None
        for m in metrics or []:
            if isinstance(m, MeanIoU):
                self.mean_iou = m
                self.metric_names.append(m.name)
            else:
                nm = m if isinstance(m, str) else getattr(m, "__name__", str(m))
                if nm not in ("dice_coef", "iou_coef"):
                    raise ValueError(f"unsupported metric {m!r}")
                self.metric_names.append(nm)

    def enable_data_parallel(self, bucket_bytes: int = 6 << 20, group=None, sync_bn: bool = False):
        """Average gradients over torch.distributed ranks each step (bucketed, overlapped).
        sync_bn: BatchNorm over the global batch (SyncBN, SURVEY 8(e) option) instead of each
        replica's shard (the reference's tf.distribute default, synchronized=False).

        With sync_bn on, every training-mode forward (train_step, engine.forward(training=True),
        model(x, training=True)) issues one blocking all-gather per BatchNorm and every backward
        one all-reduce per BatchNorm, on the main stream: ALL ranks of the group must run them
        together, in the same order, or the group hangs.  Inference (predict / evaluate,
        training=False) uses the moving statistics and issues no collective, so it may run on
        one rank alone."""
        import torch.distributed as dist
        self.bucketer = GradBucketer(self.engine.grads, bucket_bytes, group)
        self.engine.grad_hook = self.bucketer.ready
        self.engine.rank_salt = dist.get_rank(group) if dist.is_initialized() else 0
        self.engine.sync_bn = bool(sync_bn)
        self.engine.sync_group = group
        self.engine.sync_world = self.bucketer.world

    def train_step(self, x, y, global_size: Optional[int] = None) -> torch.Tensor:
        """One optimisation step; returns the device vector [loss, dice_coef, iou_coef] of this
        rank's batch (asynchronous: nothing here waits for the GPU).

        Data parallel: x is this rank's shard of a global batch of `global_size` samples (default:
        equal shards).  The shard's loss gradient is weighted n_local * world / global_size and
        the all-reduced sum scaled by 1/world, which is the gradient of the global-batch mean
        loss for any split (utils/loss.py:25-29 means over (image, class) terms)."""
        if self.optimizer is None:
            self.compile()
        x = as_device_tensor(x, self.engine.device)
        y = as_device_tensor(y, self.engine.device)
        loss_scale = 1.0
        if self.bucketer is not None and self.bucketer.world > 1:
            n_local, world = x.shape[0], self.bucketer.world
            n_global = int(global_size) if global_size else n_local * world
            if n_global < world or n_local < 1:
                raise ValueError(f"shard of {n_local} from a global batch of {n_global} over {world} ranks")
            loss_scale = n_local * world / n_global
            self.engine.sync_global_n = n_global
        caller = torch.cuda.current_stream(self.engine.device)
        main = self.engine.main
        main.wait_stream(caller)
        with torch.cuda.stream(main):
            res = self.engine.forward_train(x, y)
            if self.mean_iou is not None:  # metric only: off the critical path (the idle side stream)
                prob = self.engine.acts(x.shape[0]).prob
                self.engine.run_beside(lambda: self.mean_iou.update_state(y, prob))
            if self.loss_kind == L.LOSS_IOU:
                res = res.clone()
                res[0] = 1.0 - res[2]
            self.engine.backward(y, self.loss_kind, loss_scale)
            probe = self.dp_probe
            if probe is not None:  # bench.py's all-reduce exposure pass: main stream, end of backward
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(main)
            scale = self.bucketer.finish() if self.bucketer is not None else 1.0
            if probe is not None:  # ... and once every bucket's all-reduce has completed on it
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(main)
                probe.append((e0, e1))
            self.optimizer.apply(self.engine.params, self.engine.grads, scale)
            self.engine.params_version += 1
        caller.wait_stream(main)
        return res

    def test_step(self, x, y) -> torch.Tensor:
        x = as_device_tensor(x, self.engine.device)
        y = as_device_tensor(y, self.engine.device)
        self.engine.forward(x, training=False)
        res = self.engine.loss(y, x.shape[0])
        if self.mean_iou is not None:
            self.mean_iou.update_state(y, self.engine.acts(x.shape[0]).prob)
        if self.loss_kind == L.LOSS_IOU:
            res = res.clone()
            res[0] = 1.0 - res[2]
        return res

    def __call__(self, x, training: bool = False) -> torch.Tensor:
        x = as_device_tensor(x, self.engine.device)
        return self.engine.forward(x, training=training).clone()

    def predict(self, x, batch_size: Optional[int] = None, verbose: int = 0):
        """model.predict: numpy in -> numpy out, tensor in -> device tensor out."""
        is_np = not isinstance(x, torch.Tensor)
        xt = as_device_tensor(x, self.engine.device)
        n = xt.shape[0]
        bs = batch_size or 32
        outs = [self.engine.predict(xt[i:i + bs]) for i in range(0, n, bs)]
        out = torch.cat(outs, 0) if len(outs) > 1 else outs[0]
        return out.cpu().numpy() if is_np else out

    def _log_values(self, res: torch.Tensor, prefix: str = "") -> Dict[str, float]:
        r = res.detach().cpu().numpy()
        out = {f"{prefix}loss": float(r[0])}
        for nm in self.metric_names:
            if nm == "dice_coef":
                out[prefix + nm] = float(r[1])
            elif nm == "iou_coef":
                out[prefix + nm] = float(r[2])
        return out

    def fit(self, x=None, epochs: int = 1, steps_per_epoch: Optional[int] = None, validation_data=None,
            validation_steps: Optional[int] = None, callbacks=None, verbose: int = 1) -> History:
        """Keras fit over a generator of (image_batch, mask_batch) (scripts/train.py:308-316).
        Per-epoch logs: loss and metrics as batch means (Keras MeanMetricWrapper) and MeanIoU
        over the epoch's confusion matrix; val_* from validation_data."""
        from .callbacks import CallbackList
        if self.optimizer is None:
            self.compile()
        cbs = CallbackList(callbacks or [], self)
        hist = History()
        self.stop_training = False
        it = iter(self._prefetch(x, epochs * (steps_per_epoch or 1)))
        cbs.on_train_begin()
        for epoch in range(epochs):
            cbs.on_epoch_begin(epoch)
            if self.mean_iou is not None:
                self.mean_iou.reset_state()
            acc = None
            nsteps = 0
            t0 = time.time()
            for step in range(steps_per_epoch or 1):
                batch = next(it)
                res = self.train_step(batch[0], batch[1], getattr(batch, "global_size", None))
                acc = res.detach().clone() if acc is None else acc + res
                nsteps += 1
            logs = self._log_values(acc / nsteps)
            if self.mean_iou is not None:
                self.mean_iou.all_reduce()
                logs[self.mean_iou.name] = self.mean_iou.result()
            self.sync_bn_statistics()
            if validation_data is not None:
                logs.update(self.evaluate(validation_data, steps=validation_steps, prefix="val_"))
            for k, v in logs.items():
                hist.history.setdefault(k, []).append(v)
            hist.epoch.append(epoch)
            if verbose:
                dt = time.time() - t0
                body = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items())
                print(f"Epoch {epoch + 1}/{epochs} - {nsteps} steps - {dt:.1f}s - {body}", flush=True)
            cbs.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        cbs.on_train_end()
        if hasattr(it, "close"):
            it.close()
        return hist

    def _prefetch(self, data, limit: int):
        """Wrap a host-batch iterable in the background decoder / async H2D prefetcher.  It reads
        at most `limit` batches (the steps the caller takes), so a single-pass generator shared
        across fit / evaluate calls (a Keras-style flow) loses nothing to read-ahead."""
        from .prefetch import Prefetcher
        if isinstance(data, Prefetcher) or not hasattr(data, "__iter__"):
            return data
        return Prefetcher(data, self.engine.device, limit=limit)

    def sync_bn_statistics(self):
        """Data parallel: average the BatchNorm moving statistics over the ranks (tf.distribute
        keeps them sync-on-read MEAN; the moving update is linear, so averaging at any point
        leaves the mean's trajectory unchanged).  Called before validation and so before every
        checkpoint; a no-op on one process.  A custom loop that calls train_step directly must
        call it on EVERY rank (it is a collective) before save_weights / predict / evaluate, or
        each rank keeps its own moving statistics."""
        from .dp import average_
        if self.bucketer is not None and self.bucketer.world > 1:
            average_(self.engine.stats, self.bucketer.group)

    def evaluate(self, data, steps: Optional[int] = None, prefix: str = "") -> Dict[str, float]:
        it = iter(self._prefetch(data, steps or 1))
        if self.mean_iou is not None:
            saved = self.mean_iou.confusion.clone()
            self.mean_iou.reset_state()
        acc, n = None, 0
        for _ in range(steps or 1):
            batch = next(it)
            res = self.test_step(batch[0], batch[1])
            acc = res.detach().clone() if acc is None else acc + res
            n += 1
        if hasattr(it, "close"):
            it.close()
        logs = self._log_values(acc / n, prefix)
        if self.mean_iou is not None:
            self.mean_iou.all_reduce()
            logs[prefix + self.mean_iou.name] = self.mean_iou.result()
            self.mean_iou.confusion.copy_(saved)
        return logs

    # ------------------------------------------------------------------- weights -------
    @property
    def weights(self) -> List[str]:
        return [s.name for s in self.engine.specs]

    def get_weights(self) -> List[np.ndarray]:
        w = self.engine.get_weights_dict()
        return [w[s.name] for s in self.engine.specs]

    def set_weights(self, weights: List[np.ndarray]):
        if len(weights) != len(self.engine.specs):
            raise ValueError(f"expected {len(self.engine.specs)} arrays, got {len(weights)}")
        self.engine.set_weights_dict({s.name: w for s, w in zip(self.engine.specs, weights)})

    def save_weights(self, path: str):
        """Neutral weight file: .npz keyed by Keras weight names, Keras layouts."""
        w = self.engine.get_weights_dict()
        with open(path, "wb") as f:  # exact path (the reference's --model-out may say .h5)
            np.savez(f, **{k.replace("/", ":"): v for k, v in w.items()})

    save = save_weights

    def load_weights(self, path: str):
        with open(path, "rb") as f, np.load(f, allow_pickle=False) as z:
            self.engine.set_weights_dict({k.replace(":", "/"): z[k] for k in z.files})

    def count_params(self) -> int:
        return sum(self.engine.count_params())

    def summary(self, line_length: int = 100, print_fn=print):
        tr, nt = self.engine.count_params()
        print_fn(f'Model: "{self.name}"')
        print_fn("_" * line_length)
        print_fn(f"{'Variable':60s}{'Shape':>25s}{'Trainable':>15s}")
        print_fn("=" * line_length)
        for s in self.engine.specs:
            print_fn(f"{s.name:60s}{str(s.shape):>25s}{str(s.trainable):>15s}")
        print_fn("=" * line_length)
        print_fn(f"Total params: {tr + nt:,}")
        print_fn(f"Trainable params: {tr:,}")
        print_fn(f"Non-trainable params: {nt:,}")
        print_fn("_" * line_length)
