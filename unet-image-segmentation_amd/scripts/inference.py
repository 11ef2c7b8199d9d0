#!/usr/bin/env python3
"""Drop-in for the reference's scripts/inference.py on the MI355X engine.

Same positional/optional flags and defaults (reference scripts/inference.py:54-96), same
validation and exit codes (:207-215, :228-239), same preprocessing quirk: the image is fed as
BGR (cv2.imread order, :100-110) although training used RGB; resized bilinear to 256x256 and
scaled by 1/255; the probability map is resized back bilinear, thresholded (> threshold ->
255) and saved; the largest connected region's bounding box crops the original image.
OpenCV is not available in this image: PIL does the I/O and resizes with cv2's
INTER_LINEAR formula (half-pixel centres, no antialias); the largest external contour is
approximated by the largest 8-connected foreground component (scipy.ndimage).  This
post-processing is off the GPU path.
"""
import argparse
import os
import sys

PROJECT_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.append(PROJECT_ROOT)

import numpy as np  # noqa: E402

IMG_HEIGHT = 256
IMG_WIDTH = 256
MIN_CONTOUR_AREA = 100


def parse_args(argv=None) -> argparse.Namespace:
    parser = argparse.ArgumentParser(description="Perform segmentation and cropping using a trained U-Net model.")
    parser.add_argument("input", type=str, help="Path to the input image file.")
    parser.add_argument("--output_mask", type=str, default="./outputs_test/output_mask.png",
                        help="Output path for the predicted binary mask image (0 or 255).")
    parser.add_argument("--output_cropped", type=str, default="./outputs_test/output_cropped.png",
                        help="Output path for the cropped image based on the largest mask contour.")
    parser.add_argument("--model", type=str, default="./models/model.h5",
                        help="Path to the trained model weights file (engine .npz, Keras names).")
    parser.add_argument("--threshold", type=float, default=0.5,
                        help="Threshold value (0.0 to 1.0) to convert probability mask to binary mask.")
    parser.add_argument("--min_area", type=float, default=MIN_CONTOUR_AREA,
                        help=f"Minimum contour area threshold for cropping (default: {MIN_CONTOUR_AREA}).")
    return parser.parse_args(argv)


def resize_linear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """cv2.resize(..., INTER_LINEAR) for float images: half-pixel centres, edge clamp."""
    h, w = img.shape[:2]

    def coords(n_out, n_in):
        s = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.clip(s, 0, n_in - 1)
        i0 = np.floor(s).astype(np.int64)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, (s - i0).astype(np.float32)

    y0, y1, fy = coords(out_h, h)
    x0, x1, fx = coords(out_w, w)
    a = img[y0][:, x0]
    b = img[y0][:, x1]
    c = img[y1][:, x0]
    d = img[y1][:, x1]
    fx = fx[None, :, None] if img.ndim == 3 else fx[None, :]
    fy = fy[:, None, None] if img.ndim == 3 else fy[:, None]
    top = a + (b - a) * fx
    bot = c + (d - c) * fx
    return (top + (bot - top) * fy).astype(np.float32)


def load_and_preprocess_image(input_path, target_height, target_width):
    from PIL import Image
    try:
        rgb = np.asarray(Image.open(input_path).convert("RGB"))
    except Exception:
        print(f"Error: Could not read image from {input_path}")
        return None, None, None, None
    img_bgr = rgb[..., ::-1].copy()  # cv2.imread order (reference feeds BGR at inference)
    h, w = img_bgr.shape[:2]
    resized = resize_linear(img_bgr.astype(np.float32) / 255.0, target_height, target_width)
    return resized[None], img_bgr, h, w


def predict_mask(model, input_tensor):
    print("Running prediction...")
    try:
        pred = model.predict(input_tensor, verbose=0)
        if pred is not None and pred.ndim == 4 and pred.shape[0] == 1:
            return pred[0]
        print(f"Error: Unexpected model prediction shape: {None if pred is None else pred.shape}")
        return None
    except Exception as e:
        print(f"Error during model prediction: {e}")
        return None


def postprocess_and_save_results(prob, original_bgr, orig_h, orig_w, out_mask, out_crop, thr=0.5, min_area=100.0):
    from PIL import Image
    from scipy import ndimage
    print("Processing predicted mask...")
    resized = resize_linear(prob[..., 0], orig_h, orig_w)
    binary = (resized > thr).astype(np.uint8) * 255
    print(f"Saving binary mask to {out_mask} ...")
    if os.path.dirname(out_mask):
        os.makedirs(os.path.dirname(out_mask), exist_ok=True)
    Image.fromarray(binary).save(out_mask)
    print("Finding largest contour for cropping...")
    lab, n = ndimage.label(binary > 0, structure=np.ones((3, 3)))
    if n == 0:
        print("No contours found in the binary mask. Cropped image not saved.")
        return
    areas = ndimage.sum(np.ones_like(lab), lab, index=np.arange(1, n + 1))
    k = int(np.argmax(areas)) + 1
    area = float(areas[k - 1])
    if area <= min_area:
        print(f"Largest contour area ({area:.0f}) is below minimum threshold ({min_area:.0f}). Cropped image not saved.")
        return
    ys, xs = np.nonzero(lab == k)
    y, x, h, w = ys.min(), xs.min(), ys.max() - ys.min() + 1, xs.max() - xs.min() + 1
    print(f"Largest contour area: {area:.0f} > {min_area:.0f}. Cropping region: (x={x}, y={y}, w={w}, h={h})")
    crop = original_bgr[y:y + h, x:x + w][..., ::-1]
    print(f"Saving cropped image to {out_crop} ...")
    if os.path.dirname(out_crop):
        os.makedirs(os.path.dirname(out_crop), exist_ok=True)
    Image.fromarray(np.ascontiguousarray(crop)).save(out_crop)


def main(argv=None):
    args = parse_args(argv)
    if not os.path.isfile(args.input):
        print(f"Error: Input image not found -> {args.input}")
        sys.exit(1)
    if not os.path.isfile(args.model):
        print(f"Error: Model file not found -> {args.model}")
        sys.exit(1)
    if not (0.0 < args.threshold < 1.0):
        print(f"Error: Threshold must be between 0.0 and 1.0 -> {args.threshold}")
        sys.exit(1)
    print(f"Loading model from {args.model} ...")
    try:
        from model.u_net import U_NET
        model = U_NET((IMG_HEIGHT, IMG_WIDTH, 3), 1)
        model.load_weights(args.model)
        print("Model loaded successfully.")
    except Exception as e:
        print("\n--- Error loading model ---")
        print(f"{e}")
        sys.exit(1)
    print(f"Loading and preprocessing image: {args.input} ...")
    x, bgr, h, w = load_and_preprocess_image(args.input, IMG_HEIGHT, IMG_WIDTH)
    if x is None:
        sys.exit(1)
    prob = predict_mask(model, x)
    if prob is None:
        sys.exit(1)
    print("Postprocessing results...")
    postprocess_and_save_results(prob, bgr, h, w, args.output_mask, args.output_cropped, args.threshold,
                                 args.min_area)
    print("Inference script finished.")


if __name__ == "__main__":
    main()
