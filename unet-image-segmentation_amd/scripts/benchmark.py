#!/usr/bin/env python3
"""Drop-in for the reference's scripts/benchmark.py on the MI355X engine: dataset MeanIoU of a
trained model over MIDV-style directories (input_dir/images/**/*.tif + input_dir/ground_truth/
**/*.json holding a "quad").

Same flags and defaults (reference scripts/benchmark.py:59-93), same validation and exit codes
(:177-193, :231-233), same per-pair semantics:
  * image: BGR (cv2.imread order), /255, INTER_LINEAR to 256x256            (:95-110)
  * truth: the quad filled (drawContours FILLED) at the companion image's original size,
    INTER_NEAREST to 256x256, > 128                                          (:112-157)
  * prediction: model.predict, p > pred_threshold                             (:254-260)
  * per-sample IoU (I + eps)/(T + P - I + eps) in float32, eps = 1e-7; files below
    --iou_threshold are listed, sorted by score, and written to --low_score_log as
    "FileID,MeanIoU_Score"                                                    (:159-170, :264-299)
  * MeanIoU(num_classes=2) over all pairs (keras.metrics.MeanIoU)             (:237, :269, :277)
The forward runs on the GPU in batches (inference BatchNorm uses the moving statistics, so a
sample's output does not depend on its batch); the confusion counts accumulate on the device
(unet_meaniou_update).  OpenCV steps are restated in unet_amd/imageproc.py.
"""
import argparse
import json
import os
import sys
import time
from glob import glob
from typing import Dict, List, Optional, Tuple

PROJECT_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if PROJECT_ROOT not in sys.path:
    sys.path.append(PROJECT_ROOT)

import numpy as np  # noqa: E402

from unet_amd.imageproc import fill_quad, resize_linear, resize_nearest  # noqa: E402

IMG_HEIGHT = 256
IMG_WIDTH = 256
SMOOTH = 1e-7  # K.epsilon()
BATCH = 16


def parse_args(argv=None) -> argparse.Namespace:
    parser = argparse.ArgumentParser(description="Benchmark a U-Net segmentation model using JSON ground truth.")
    parser.add_argument("input_dir", type=str,
                        help="Top-level directory containing 'images/' and 'ground_truth/' subfolders.")
    parser.add_argument("--model", type=str, default="./models/model.h5",
                        help="Path to the trained model weights file (engine .npz, Keras names).")
    parser.add_argument("--iou_threshold", type=float, default=0.9,
                        help="Log filenames where the sample's MeanIoU is BELOW this threshold.")
    parser.add_argument("--pred_threshold", type=float, default=0.5,
                        help="Threshold (0-1) to convert model's probability prediction to a binary mask.")
    parser.add_argument("--low_score_log", type=str, default=None,
                        help="Optional file path to save the list of files scoring below the iou_threshold.")
    return parser.parse_args(argv)


def _read_bgr(path: str) -> Optional[np.ndarray]:
    from PIL import Image
    try:
        with Image.open(path) as im:
            return np.asarray(im.convert("RGB"))[..., ::-1]
    except Exception:
        return None


def load_image_for_predict(img_path: str) -> Optional[np.ndarray]:
    """(1, 256, 256, 3) float32: BGR, /255, INTER_LINEAR (reference :95-110)."""
    bgr = _read_bgr(img_path)
    if bgr is None:
        print(f"Warning: Could not read image: {img_path}. Skipping.")
        return None
    return resize_linear(bgr.astype(np.float32) / 255.0, IMG_HEIGHT, IMG_WIDTH)[None]


def build_mask_from_quad(json_path: str, target_height: int, target_width: int) -> Optional[np.ndarray]:
    """(1, H, W, 1) uint8 {0, 1} truth mask from the JSON quad (reference :112-157)."""
    from PIL import Image
    try:
        with open(json_path, "r") as f:
            data = json.load(f)
        quad = data.get("quad", [])
        orig_h = orig_w = -1
        for ext in (".tif", ".png", ".jpg"):
            p = json_path.replace("/ground_truth/", "/images/").replace(".json", ext)
            if os.path.exists(p):
                with Image.open(p) as im:
                    orig_w, orig_h = im.size
                break
        if orig_h <= 0 or orig_w <= 0:
            print(f"Warning: Could not determine original dimensions for mask from {json_path}. "
                  f"Using default large canvas (2048x2048).")
            orig_h, orig_w = 2048, 2048
        mask = np.zeros((orig_h, orig_w), dtype=np.uint8)
        if quad:
            fill_quad(mask, np.asarray(quad, dtype=np.int64).reshape(-1, 2), 255)
        binary = (resize_nearest(mask, target_height, target_width) > 128).astype(np.uint8)
        return binary[None, :, :, None]
    except FileNotFoundError:
        print(f"Error: JSON file not found: {json_path}")
        return None
    except Exception as e:
        print(f"Error processing JSON/Mask {json_path}: {e}")
        return None


def calculate_sample_iou(y_true: np.ndarray, y_pred: np.ndarray, smooth: float = SMOOTH) -> float:
    """(I + smooth) / (T + P - I + smooth) in float32 (reference :159-170)."""
    t = y_true.squeeze().astype(np.float32)
    p = y_pred.squeeze().astype(np.float32)
    inter = np.float32((t * p).sum(dtype=np.float32))
    st, sp = np.float32(t.sum(dtype=np.float32)), np.float32(p.sum(dtype=np.float32))
    union = st + sp - inter
    return float((inter + np.float32(smooth)) / (union + np.float32(smooth)))


def find_pairs(images_root: str, gtruth_root: str) -> Tuple[List[Dict], int]:
    image_files = sorted(glob(os.path.join(images_root, "**", "*.tif"), recursive=True))
    print(f"Found {len(image_files)} '.tif' images.")
    pairs, skipped = [], 0
    for img_path in image_files:
        base = os.path.splitext(os.path.relpath(img_path, images_root))[0]
        json_path = os.path.join(gtruth_root, base + ".json")
        if os.path.isfile(json_path):
            pairs.append({"image": img_path, "json": json_path, "id": base})
        else:
            print(f"Warning: No corresponding JSON found for {img_path}. Skipping.")
            skipped += 1
    return pairs, skipped


def evaluate(model, pairs: List[Dict], pred_threshold: float, iou_threshold: float, device=None):
    """Overall MeanIoU(2) and the (file_id, sample IoU) pairs below iou_threshold."""
    import torch
    from unet_amd.metrics import MeanIoU
    miou = MeanIoU(num_classes=2, name="overall_mean_iou", threshold=pred_threshold, device=device)
    low: List[Tuple[str, float]] = []
    batch: List[Tuple[str, np.ndarray, np.ndarray]] = []

    def flush():
        if not batch:
            return
        x = np.concatenate([b[1] for b in batch])
        yt = np.concatenate([b[2] for b in batch]).astype(np.float32)
        prob = model.predict(x) if device is None else model.predict(torch.as_tensor(x, device=device))
        prob_t = torch.as_tensor(prob, device=miou.device)
        miou.update_state(torch.as_tensor(yt, device=miou.device), prob_t)  # p > thr on the device
        pred = (prob_t > pred_threshold).to(torch.uint8).cpu().numpy()
        for (fid, _, t), p in zip(batch, pred):
            s = calculate_sample_iou(t, p)
            if s < iou_threshold:
                low.append((fid, s))
                print(f"\nBelow threshold (IoU={s:.3f}): {fid}")
        batch.clear()

    for i, pair in enumerate(pairs):
        print(f"\rProcessing [{i + 1}/{len(pairs)}]: {pair['id']}", end="")
        img = load_image_for_predict(pair["image"])
        truth = build_mask_from_quad(pair["json"], IMG_HEIGHT, IMG_WIDTH)
        if img is None or truth is None:
            print(f"\nSkipping pair due to loading error: {pair['id']}")
            continue
        batch.append((pair["id"], img, truth))
        if len(batch) == BATCH:
            flush()
    flush()
    return miou.result(), low


def main(argv=None):
    args = parse_args(argv)
    start = time.time()
    if not os.path.isdir(args.input_dir):
        print(f"Error: Input directory not found -> {args.input_dir}")
        sys.exit(1)
    images_root = os.path.join(args.input_dir, "images")
    gtruth_root = os.path.join(args.input_dir, "ground_truth")
    if not (os.path.isdir(images_root) and os.path.isdir(gtruth_root)):
        print(f"Error: '{images_root}' or '{gtruth_root}' not found.")
        sys.exit(1)
    if not os.path.isfile(args.model):
        print(f"Error: Model file not found -> {args.model}")
        sys.exit(1)
    if not 0.0 <= args.pred_threshold <= 1.0:
        print(f"Error: Prediction threshold must be between 0.0 and 1.0 -> {args.pred_threshold}")
        sys.exit(1)
    if not 0.0 <= args.iou_threshold <= 1.0:
        print(f"Error: IoU threshold must be between 0.0 and 1.0 -> {args.iou_threshold}")
        sys.exit(1)
    print(f"Loading model: {args.model} ...")
    try:
        from model.u_net import U_NET
        model = U_NET((IMG_HEIGHT, IMG_WIDTH, 3), 1)
        model.load_weights(args.model)
        print("Model loaded successfully.")
    except Exception as e:
        print("\n--- Error loading model ---")
        print(f"{e}")
        print("---------------------------\n")
        sys.exit(1)
    print("Finding image and ground truth pairs...")
    pairs, skipped = find_pairs(images_root, gtruth_root)
    if not pairs:
        print("Error: No valid image/JSON pairs found. Check dataset structure and file extensions.")
        sys.exit(1)
    print(f"Prepared {len(pairs)} image/JSON pairs for evaluation ({skipped} images skipped).")
    print(f"Evaluating model (Prediction Threshold: {args.pred_threshold:.2f})...")
    final, low = evaluate(model, pairs, args.pred_threshold, args.iou_threshold)
    print("\nEvaluation complete.")
    print(f"\n{'=' * 30}")
    print(f"Overall Mean IoU: {final:.4f}")
    print(f"{'=' * 30}")
    if low:
        print(f"\nFiles scoring below IoU threshold ({args.iou_threshold:.2f}):")
        low.sort(key=lambda t: t[1])
        for fid, score in low:
            print(f"  - IoU: {score:.4f} | File: {fid}")
        if args.low_score_log:
            print(f"\nSaving low score list to: {args.low_score_log}")
            try:
                d = os.path.dirname(args.low_score_log)
                if d:
                    os.makedirs(d, exist_ok=True)
                with open(args.low_score_log, "w") as f:
                    f.write("FileID,MeanIoU_Score\n")
                    for fid, score in low:
                        f.write(f"{fid},{score:.4f}\n")
            except Exception as e:
                print(f"Error saving low score log: {e}")
    else:
        print(f"\nNo files scored below the IoU threshold ({args.iou_threshold:.2f}).")
    print(f"\nTotal benchmark time: {time.time() - start:.2f} seconds.")
    print("Benchmark script finished.")


if __name__ == "__main__":
    main()
