"""The Keras callbacks scripts/train.py wires into model.fit (:273-304), on the engine.

ModelCheckpoint (save_best_only on val_mean_io_u), EarlyStopping (patience 10,
restore_best_weights), ReduceLROnPlateau (factor 0.2, patience 3, min_lr 1e-6).  TensorBoard
(:299-302) has no equivalent here: CSVLogger-style JSON lines are written instead.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import numpy as np


class Callback:
    model = None

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass


class CallbackList:
    def __init__(self, callbacks: List[Callback], model):
        self.callbacks = list(callbacks)
        for c in self.callbacks:
            c.set_model(model)

    def on_train_begin(self):
        for c in self.callbacks:
            c.on_train_begin()

    def on_train_end(self):
        for c in self.callbacks:
            c.on_train_end()

    def on_epoch_begin(self, epoch):
        for c in self.callbacks:
            c.on_epoch_begin(epoch)

    def on_epoch_end(self, epoch, logs):
        for c in self.callbacks:
            c.on_epoch_end(epoch, logs)


def _better(mode: str, cur: float, best: float, min_delta: float = 0.0) -> bool:
    if mode == "min":
        return cur < best - min_delta
    return cur > best + min_delta


class _Monitor(Callback):
    def __init__(self, monitor: str, mode: str):
        if mode == "auto":
            mode = "min" if "loss" in monitor else "max"
        self.monitor = monitor
        self.mode = mode
        self.best = np.inf if mode == "min" else -np.inf

    def _get(self, logs: Dict[str, float]) -> Optional[float]:
        v = (logs or {}).get(self.monitor)
        return None if v is None else float(v)


class ModelCheckpoint(_Monitor):
    def __init__(self, filepath: str, monitor: str = "val_loss", mode: str = "auto", save_best_only: bool = False,
                 save_weights_only: bool = False, verbose: int = 0):
        super().__init__(monitor, mode)
        self.filepath = filepath
        self.save_best_only = save_best_only
        self.verbose = verbose

    def on_epoch_end(self, epoch, logs=None):
        cur = self._get(logs)
        if self.save_best_only:
            if cur is None or not _better(self.mode, cur, self.best):
                if self.verbose and cur is not None:
                    print(f"\nEpoch {epoch + 1}: {self.monitor} did not improve from {self.best:.5f}")
                return
            if self.verbose:
                print(f"\nEpoch {epoch + 1}: {self.monitor} improved from {self.best:.5f} to {cur:.5f}, "
                      f"saving model to {self.filepath}")
            self.best = cur
        d = os.path.dirname(self.filepath)
        if d:
            os.makedirs(d, exist_ok=True)
        self.model.save_weights(self.filepath)


class EarlyStopping(_Monitor):
    def __init__(self, monitor: str = "val_loss", patience: int = 0, mode: str = "auto",
                 restore_best_weights: bool = False, verbose: int = 0, min_delta: float = 0.0):
        super().__init__(monitor, mode)
        self.patience = patience
        self.restore_best_weights = restore_best_weights
        self.verbose = verbose
        self.min_delta = min_delta
        self.wait = 0
        self.stopped_epoch = 0
        self.best_weights = None

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.stopped_epoch = 0
        self.best = np.inf if self.mode == "min" else -np.inf
        self.best_weights = None

    def on_epoch_end(self, epoch, logs=None):
        cur = self._get(logs)
        if cur is None:
            return
        if _better(self.mode, cur, self.best, self.min_delta):
            self.best = cur
            self.wait = 0
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
            return
        self.wait += 1
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            self.model.stop_training = True
            if self.restore_best_weights and self.best_weights is not None:
                if self.verbose:
                    print("Restoring model weights from the end of the best epoch.")
                self.model.set_weights(self.best_weights)

    def on_train_end(self, logs=None):
        if self.stopped_epoch > 0 and self.verbose:
            print(f"Epoch {self.stopped_epoch + 1}: early stopping")


class ReduceLROnPlateau(_Monitor):
    def __init__(self, monitor: str = "val_loss", factor: float = 0.1, patience: int = 10, mode: str = "auto",
                 min_lr: float = 0.0, verbose: int = 0, min_delta: float = 1e-4, cooldown: int = 0):
        super().__init__(monitor, mode)
        if factor >= 1.0:
            raise ValueError("ReduceLROnPlateau does not support a factor >= 1.0")
        self.factor = factor
        self.patience = patience
        self.min_lr = min_lr
        self.verbose = verbose
        self.min_delta = min_delta
        self.cooldown = cooldown
        self.cooldown_counter = 0
        self.wait = 0

    def on_epoch_end(self, epoch, logs=None):
        cur = self._get(logs)
        if cur is None:
            return
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if _better(self.mode, cur, self.best, self.min_delta):
            self.best = cur
            self.wait = 0
        elif self.cooldown_counter <= 0:
            self.wait += 1
            if self.wait >= self.patience:
                opt = self.model.optimizer
                old = float(opt.learning_rate)
                if old > self.min_lr:
                    new = max(old * self.factor, self.min_lr)
                    opt.learning_rate = new
                    if self.verbose:
                        print(f"\nEpoch {epoch + 1}: ReduceLROnPlateau reducing learning rate to {new}.")
                    self.cooldown_counter = self.cooldown
                    self.wait = 0


class JSONLogger(Callback):
    """Stands in for TensorBoard(log_dir): one JSON line of logs per epoch."""

    def __init__(self, log_dir: str):
        self.log_dir = log_dir

    def on_epoch_end(self, epoch, logs=None):
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, "history.jsonl"), "a") as f:
            f.write(json.dumps({"epoch": epoch + 1, **{k: float(v) for k, v in (logs or {}).items()}}) + "\n")
