"""CPU restatements of the reference CLIs' OpenCV steps (unet_amd/imageproc.py).

Pinned by the reference's own outputs: samples/usage/<name>/output_mask.png is the binary mask
the reference's inference.py saved for samples/test_images/<name>.png, and output_cropped.png
the crop it then cut with cv2.findContours / contourArea / boundingRect.  For chile_id_card the
crop of our largest external contour is pixel-identical to the reference's file; for
brazil_passport the reference's crop has exactly our bounding-box size but its pixels do not
come from the shipped test image (no offset within the image reproduces them), so only the box
size is pinned there.  cv2 is not importable here: the remaining known-answer cases follow
OpenCV's documented conventions (parity unpinned beyond the samples)."""
import os

import numpy as np
import pytest
from PIL import Image

from unet_amd.imageproc import (bounding_rect, contour_area, external_contours, fill_quad,
                                largest_external_contour, resize_linear, resize_nearest)

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "samples")


def _png(p, mode):
    with Image.open(p) as im:
        return np.asarray(im.convert(mode))


def test_reference_sample_crop_chile_pixel_exact():
    mask = _png(os.path.join(HERE, "usage", "chile_id_card_output_mask.png"), "L")
    img = _png(os.path.join(HERE, "chile_id_card.png"), "RGB")
    ref = _png(os.path.join(HERE, "usage", "chile_id_card_output_cropped.png"), "RGB")
    area, (x, y, w, h) = largest_external_contour(mask > 0)
    assert area > 100
    assert np.array_equal(img[y:y + h, x:x + w], ref)


def test_reference_sample_crop_brazil_box_size():
    mask = _png(os.path.join(HERE, "usage", "brazil_passport_output_mask.png"), "L")
    ref = _png(os.path.join(HERE, "usage", "brazil_passport_output_cropped.png"), "RGB")
    area, (x, y, w, h) = largest_external_contour(mask > 0)
    assert (h, w) == ref.shape[:2]


def test_contour_area_rectangle_and_degenerates():
    m = np.zeros((10, 12), np.uint8)
    m[2:6, 3:9] = 1
    (c,) = external_contours(m)
    assert contour_area(c) == (6 - 1) * (4 - 1)
    assert bounding_rect(c) == (3, 2, 6, 4)
    p = np.zeros((5, 5), np.uint8)
    p[2, 2] = 1
    (c1,) = external_contours(p)
    assert contour_area(c1) == 0 and bounding_rect(c1) == (2, 2, 1, 1)
    ln = np.zeros((5, 9), np.uint8)
    ln[2, 1:8] = 1
    assert contour_area(external_contours(ln)[0]) == 0


def test_external_only_and_holes_included():
    m = np.zeros((12, 12), np.uint8)
    m[1:11, 1:11] = 1
    m[3:9, 3:9] = 0          # hole
    m[5:7, 5:7] = 1          # island inside the hole: not an external contour
    cs = external_contours(m)
    assert len(cs) == 1
    assert contour_area(cs[0]) == 9 * 9   # the hole does not reduce the outer contour's area


def test_largest_picks_by_area_not_pixel_count():
    m = np.zeros((20, 40), np.uint8)
    m[2:4, 2:38] = 1     # 2 x 36 = 72 pixels, area 1 x 35 = 35
    m[8:15, 5:12] = 1    # 7 x 7 = 49 pixels, area 36
    area, box = largest_external_contour(m)
    assert area == 36 and box == (5, 8, 7, 7)
    assert largest_external_contour(np.zeros((4, 4))) is None


def test_diagonal_component_is_one_8_connected_contour():
    m = np.eye(6, dtype=np.uint8)
    cs = external_contours(m)
    assert len(cs) == 1 and bounding_rect(cs[0]) == (0, 0, 6, 6)


def test_resize_nearest_floor_rule():
    a = np.arange(10, dtype=np.uint8)[None, :].repeat(2, 0)
    r = resize_nearest(a, 2, 4)
    assert r[0].tolist() == [0, 2, 5, 7]   # floor(i * 10 / 4)


def test_resize_linear_half_pixel_centres():
    a = np.array([[0.0, 1.0, 2.0, 3.0]], np.float32)
    r = resize_linear(a, 1, 2)
    assert np.allclose(r, [[0.5, 2.5]])
    up = resize_linear(np.array([[0.0, 1.0]], np.float32), 1, 4)
    assert np.allclose(up, [[0.0, 0.25, 0.75, 1.0]])


def test_fill_quad_axis_aligned_and_triangle():
    m = np.zeros((10, 10), np.uint8)
    fill_quad(m, [[2, 1], [7, 1], [7, 5], [2, 5]])
    exp = np.zeros_like(m)
    exp[1:6, 2:8] = 255
    assert np.array_equal(m, exp)
    t = np.zeros((8, 8), np.uint8)
    fill_quad(t, [[0, 0], [6, 0], [0, 6]], 1)
    # every pixel on or below the anti-diagonal x + y <= 6
    yy, xx = np.mgrid[0:8, 0:8]
    assert np.array_equal(t.astype(bool), (xx + yy <= 6))
