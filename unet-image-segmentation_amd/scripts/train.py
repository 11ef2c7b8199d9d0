#!/usr/bin/env python3
"""Drop-in for the reference's scripts/train.py on the MI355X engine.

Same flags and defaults (reference scripts/train.py:71-117): --epochs 30 --batch-size 2
--learning-rate 2e-3 --weight-decay 1e-4 --model-out ./models/model.h5; same dataset layout
(dataset/train/{train,val}_{frames,masks}/image), same seed (2301), rescale 1/255,
synchronised horizontal flips for training, same callbacks (ModelCheckpoint on
val_mean_io_u, EarlyStopping patience 10, ReduceLROnPlateau factor 0.2 patience 3).
Extras: --synthetic N (no dataset needed), data-parallel via torchrun env (one process per
GPU, each rank takes its shard of every global batch).  The model file is the engine's
neutral .npz weight file (Keras names and layouts), whatever the extension.
"""
import argparse
import os
import sys
import time

PROJECT_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if PROJECT_ROOT not in sys.path:
    sys.path.append(PROJECT_ROOT)

import numpy as np  # noqa: E402

from model.u_net import U_NET  # noqa: E402
from utils.loss import dice_loss  # noqa: E402
from utils.metrics import dice_coef  # noqa: E402

DEFAULT_EPOCHS = 30
DEFAULT_BATCHSIZE = 2
DEFAULT_LR = 2e-3
DEFAULT_WEIGHT_DECAY = 1e-4
DEFAULT_MODEL_OUT = "./models/model.h5"
SEED = 2301
TRAIN_FRAMES_DIR = "dataset/train/train_frames/image"
TRAIN_MASKS_DIR = "dataset/train/train_masks/image"
VAL_FRAMES_DIR = "dataset/train/val_frames/image"
VAL_MASKS_DIR = "dataset/train/val_masks/image"
IMAGE_HEIGHT = 256
IMAGE_WIDTH = 256
IMAGE_CHANNELS = 3
MODEL_INPUT_SHAPE = (IMAGE_HEIGHT, IMAGE_WIDTH, IMAGE_CHANNELS)
TARGET_SIZE = (IMAGE_HEIGHT, IMAGE_WIDTH)
NUM_CLASSES = 1


def parse_args(argv=None) -> argparse.Namespace:
    parser = argparse.ArgumentParser(description="Train a U-Net model for binary segmentation using AdamW.")
    parser.add_argument("--epochs", type=int, default=DEFAULT_EPOCHS,
                        help=f"Number of training epochs (default: {DEFAULT_EPOCHS}).")
    parser.add_argument("--batch-size", type=int, default=DEFAULT_BATCHSIZE,
                        help=f"Batch size (default: {DEFAULT_BATCHSIZE}).")
    parser.add_argument("--learning-rate", type=float, default=DEFAULT_LR,
                        help=f"Initial learning rate for AdamW optimizer (default: {DEFAULT_LR}).")
    parser.add_argument("--weight-decay", type=float, default=DEFAULT_WEIGHT_DECAY,
                        help=f"Weight decay for AdamW optimizer (default: {DEFAULT_WEIGHT_DECAY}).")
    parser.add_argument("--model-out", type=str, default=DEFAULT_MODEL_OUT,
                        help=f"File path to save the best trained model (default: {DEFAULT_MODEL_OUT}).")
    parser.add_argument("--synthetic", type=int, default=0,
                        help="Use N synthetic image/mask pairs instead of the dataset directories.")
    parser.add_argument("--dataset-root", type=str, default=".", help="Directory holding dataset/.")
    return parser.parse_args(argv)


def count_samples(train, val, root="."):
    """Sample counts from the loaders, falling back to listing the frame directories when a loader
    cannot report them (reference scripts/train.py:237-249).  Exits 1 if neither works."""
    try:
        n_train, n_val = train.samples, val.samples
        print(f"Found {n_train} training samples and {n_val} validation samples.")
    except Exception as e:
        print(f"Warning: Could not read sample count from generators ({e}). Falling back to file listing.")
        try:
            n_train = len(os.listdir(os.path.join(root, TRAIN_FRAMES_DIR)))
            n_val = len(os.listdir(os.path.join(root, VAL_FRAMES_DIR)))
            print(f"(Fallback) Counted {n_train} train files, {n_val} val files.")
        except FileNotFoundError as fe:
            print(f"Error counting files: {fe}. Please check dataset paths.")
            sys.exit(1)
    return n_train, n_val


def training_summary(history, early_stopping, monitor_metric, monitor_mode, epochs):
    """The report after model.fit (reference scripts/train.py:317-331): the early-stopping epoch
    if it triggered, the best monitored score, and the epoch it came from with the reference's
    own arithmetic (stopped epoch - patience when early stopping fired, else argmax + 1 for a
    'max' monitor, else 'N/A')."""
    lines = []
    best = np.inf if monitor_mode == "min" else -np.inf
    stopped = epochs
    fired = early_stopping is not None and early_stopping.stopped_epoch > 0
    if fired:
        stopped = early_stopping.stopped_epoch + 1
        lines.append(f"Early stopping triggered at epoch {stopped}")
        best = early_stopping.best
    else:
        scores = history.history.get(monitor_metric)
        if scores:
            best = min(scores) if monitor_mode == "min" else max(scores)
    if fired:
        at = stopped - early_stopping.patience
    elif monitor_mode == "max" and monitor_metric in history.history:
        at = int(np.argmax(history.history[monitor_metric])) + 1
    else:
        at = "N/A"
    lines.append(f"Best monitored score ({monitor_metric}): {best:.4f} (from epoch {at})")
    return lines


def main(argv=None):
    args = parse_args(argv)
    from unet_amd.callbacks import EarlyStopping, JSONLogger, ModelCheckpoint, ReduceLROnPlateau
    from unet_amd.data import PairLoader, synthetic_pairs
    from unet_amd.dp import init_from_env
    from unet_amd.metrics import MeanIoU
    from unet_amd.optim import AdamW

    rank, world, local = init_from_env()
    np.random.seed(SEED)
    say = print if rank == 0 else (lambda *a, **k: None)
    say("\n--- Training Configuration ---")
    say(f"Epochs        : {args.epochs}")
    say(f"Batch Size    : {args.batch_size}")
    say(f"Learning Rate : {args.learning_rate}")
    say(f"Weight Decay  : {args.weight_decay} (for AdamW)")
    say(f"Model Output  : {args.model_out}")
    say(f"Input Shape   : {MODEL_INPUT_SHAPE}")
    say(f"Target Size   : {TARGET_SIZE}")
    say(f"Seed          : {SEED}")
    say(f"GPUs          : {world} (data parallel)")
    say("------------------------------\n")
    if args.batch_size < world:  # every data-parallel rank needs at least one sample per step
        print(f"Error: --batch-size {args.batch_size} is smaller than the {world} data-parallel ranks.")
        sys.exit(1)

    say("Setting up Data Generators...")
    try:
        if args.synthetic:
            train = synthetic_pairs(args.synthetic, TARGET_SIZE, args.batch_size, SEED, shuffle=True,
                                    rank=rank, world=world)
            val = synthetic_pairs(max(args.synthetic // 5, args.batch_size), TARGET_SIZE, args.batch_size, SEED + 1,
                                  shuffle=False, rank=rank, world=world)
        else:
            root = args.dataset_root
            train = PairLoader(os.path.join(root, TRAIN_FRAMES_DIR), os.path.join(root, TRAIN_MASKS_DIR),
                               TARGET_SIZE, args.batch_size, SEED, shuffle=True, horizontal_flip=True,
                               rank=rank, world=world)
            val = PairLoader(os.path.join(root, VAL_FRAMES_DIR), os.path.join(root, VAL_MASKS_DIR), TARGET_SIZE,
                             args.batch_size, SEED, shuffle=False, horizontal_flip=False, rank=rank, world=world)
        say("Data Generators created successfully.")
    except Exception as e:  # reference: print + exit(1) (train.py:208-217)
        print("\n--- Error initializing ImageDataGenerator ---")
        print(f"{e}")
        print("Please ensure dataset directories exist and follow the expected structure:")
        print(f"  Train Images: {TRAIN_FRAMES_DIR}/..")
        print(f"  Train Masks : {TRAIN_MASKS_DIR}/..")
        print(f"  Val Images  : {VAL_FRAMES_DIR}/..")
        print(f"  Val Masks   : {VAL_MASKS_DIR}/..")
        print("-------------------------------------------\n")
        sys.exit(1)

    say("Building U-Net model...")
    model = U_NET(input_size=MODEL_INPUT_SHAPE, num_classes=NUM_CLASSES, device=f"cuda:{local}")
    say("Compiling model with AdamW optimizer and Dice loss...")
    model.compile(optimizer=AdamW(learning_rate=args.learning_rate, weight_decay=args.weight_decay),
                  loss=dice_loss, metrics=[MeanIoU(num_classes=2, name="mean_io_u", device=f"cuda:{local}"),
                                           dice_coef])
    if world > 1:
        model.enable_data_parallel()
    if rank == 0:
        model.summary(line_length=100)

    if rank == 0:
        n_train, n_val = count_samples(train, val, args.dataset_root)
    else:
        n_train, n_val = train.samples, val.samples
    if n_train == 0 or n_val == 0:
        print("Error: No training or validation images found/loaded. Check dataset paths and contents.")
        sys.exit(1)
    steps_per_epoch = max(1, n_train // args.batch_size)
    validation_steps = max(1, n_val // args.batch_size)
    say(f"Steps per epoch: {steps_per_epoch}, Validation steps: {validation_steps}")
    if n_train < args.batch_size:
        say(f"Warning: Training dataset size ({n_train}) < batch size ({args.batch_size}).")
    if n_val < args.batch_size:
        say(f"Warning: Validation dataset size ({n_val}) < batch size ({args.batch_size}).")

    monitor_metric, monitor_mode = "val_mean_io_u", "max"
    say(f"Setting up Callbacks - Monitoring: '{monitor_metric}' (mode: {monitor_mode})")
    model_dir = os.path.dirname(args.model_out)
    if model_dir:
        os.makedirs(model_dir, exist_ok=True)
        say(f"Ensured model save directory exists: {model_dir}")
    early_stopping = EarlyStopping(monitor=monitor_metric, patience=10, mode=monitor_mode, restore_best_weights=True,
                                   verbose=1 if rank == 0 else 0)
    callbacks = [early_stopping,
                 ReduceLROnPlateau(monitor=monitor_metric, factor=0.2, patience=3, mode=monitor_mode, min_lr=1e-6,
                                   verbose=1 if rank == 0 else 0)]
    if rank == 0:
        callbacks.insert(0, ModelCheckpoint(filepath=args.model_out, monitor=monitor_metric, mode=monitor_mode,
                                            save_best_only=True, verbose=1))
        log_dir = os.path.join("./logs", time.strftime("%Y%m%d_%H%M%S"))
        say(f"TensorBoard logs will be saved to: {log_dir}")
        callbacks.append(JSONLogger(log_dir))

    say(f"\n--- Starting Training ({args.epochs} epochs) ---")
    try:
        history = model.fit(train, epochs=args.epochs, steps_per_epoch=steps_per_epoch, validation_data=val,
                            validation_steps=validation_steps, callbacks=callbacks, verbose=1 if rank == 0 else 0)
        say("\n--- Training complete ---")
        for line in training_summary(history, early_stopping, monitor_metric, monitor_mode, args.epochs):
            say(line)
        say(f"Best model saved to: {args.model_out}")
    except KeyboardInterrupt:
        print("\n--- Training interrupted by user ---")
        print(f"Model state might not be saved correctly to {args.model_out} unless a checkpoint occurred.")
        sys.exit(1)
    except Exception as e:
        print("\n--- Error during model training ---")
        print(f"{e}")
        import traceback
        traceback.print_exc()
        print("-----------------------------------\n")
        sys.exit(1)


if __name__ == "__main__":
    main()
