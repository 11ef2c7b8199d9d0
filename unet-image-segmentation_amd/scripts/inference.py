#!/usr/bin/env python3
"""Drop-in for the reference's scripts/inference.py on the MI355X engine.

Same positional/optional flags and defaults (reference scripts/inference.py:54-96), same
validation and exit codes (:207-215, :228-239), same preprocessing quirk: the image is fed as
BGR (cv2.imread order, :100-110) although training used RGB; resized bilinear to 256x256 and
scaled by 1/255; the probability map is resized back bilinear, thresholded (> threshold ->
255) and saved; the bounding box of the external contour of largest cv2.contourArea crops
the original image.  OpenCV is not available in this image: PIL does the I/O, and
unet_amd/imageproc.py restates cv2.resize INTER_LINEAR (half-pixel centres, no antialias) and
findContours(RETR_EXTERNAL) + contourArea (shoelace area of the traced boundary-pixel chain,
holes included) + boundingRect.  The reference's own sample output (samples/usage) pins the
crop (tests/test_imageproc.py).  This post-processing is off the GPU path.
"""
import argparse
import os
import sys

PROJECT_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.append(PROJECT_ROOT)

import numpy as np  # noqa: E402

from unet_amd.imageproc import largest_external_contour, resize_linear  # noqa: E402

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
    print("Processing predicted mask...")
    resized = resize_linear(prob[..., 0], orig_h, orig_w)
    binary = (resized > thr).astype(np.uint8) * 255
    print(f"Saving binary mask to {out_mask} ...")
    if os.path.dirname(out_mask):
        os.makedirs(os.path.dirname(out_mask), exist_ok=True)
    Image.fromarray(binary).save(out_mask)
    print("Finding largest contour for cropping...")
    best = largest_external_contour(binary)
    if best is None:
        print("No contours found in the binary mask. Cropped image not saved.")
        return
    area, (x, y, w, h) = best
    if not area > min_area:
        print(f"Largest contour area ({area:.0f}) is below minimum threshold ({min_area:.0f}). Cropped image not saved.")
        return
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
