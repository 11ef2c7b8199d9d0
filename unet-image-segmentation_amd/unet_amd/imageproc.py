"""Host-side image steps of the reference CLIs (OpenCV there; not importable here), restated in
NumPy.  They are CPU pre/post-processing around the GPU forward, off the hot path:

  resize_linear     cv2.resize(float image, INTER_LINEAR)   scripts/inference.py:105-108, :147-149,
                                                            scripts/benchmark.py:105
  resize_nearest    cv2.resize(uint8 mask, INTER_NEAREST)    scripts/benchmark.py:147
  fill_quad         cv2.drawContours(mask, [quad], -1, 255, FILLED)   scripts/benchmark.py:135-142
  external_contours cv2.findContours(binary, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)
                    + cv2.contourArea + cv2.boundingRect    scripts/inference.py:173-187

Conventions follow OpenCV's documented behaviour: INTER_LINEAR samples at half-pixel centres
with edge clamping; INTER_NEAREST takes source index floor(dst * src/dst); a contour is the
chain of boundary pixel centres of an 8-connected foreground component found by Suzuki-Abe
outer-border following, its area the shoelace area of that chain (so a filled w x h rectangle
has area (w-1)(h-1), holes are included, a single pixel or a line has area 0); RETR_EXTERNAL
keeps only components not nested inside another component's hole.  The outputs the reference
itself produced for its sample images pin the contour crop (tests/test_imageproc.py).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

# 8 neighbours in OpenCV's chain-code order: 0 = right, then counter-clockwise on screen
# (image rows grow downwards): right, up-right, up, up-left, left, down-left, down, down-right
_DIRS = ((0, 1), (-1, 1), (-1, 0), (-1, -1), (0, -1), (1, -1), (1, 0), (1, 1))


def resize_linear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """cv2.resize(img, (out_w, out_h), interpolation=INTER_LINEAR) for float images."""
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


def resize_nearest(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """cv2.resize(img, (out_w, out_h), interpolation=INTER_NEAREST): src = floor(dst * src/dst)."""
    h, w = img.shape[:2]
    ys = np.minimum(np.floor(np.arange(out_h) * (h / out_h)).astype(np.int64), h - 1)
    xs = np.minimum(np.floor(np.arange(out_w) * (w / out_w)).astype(np.int64), w - 1)
    return img[ys][:, xs]


def _line8(mask: np.ndarray, p0, p1, value) -> None:
    """8-connected Bresenham segment between integer points (x, y), clipped to the image."""
    x0, y0 = int(p0[0]), int(p0[1])
    x1, y1 = int(p1[0]), int(p1[1])
    dx, dy = abs(x1 - x0), -abs(y1 - y0)
    sx, sy = (1 if x0 < x1 else -1), (1 if y0 < y1 else -1)
    err = dx + dy
    H, W = mask.shape[:2]
    while True:
        if 0 <= y0 < H and 0 <= x0 < W:
            mask[y0, x0] = value
        if x0 == x1 and y0 == y1:
            return
        e2 = 2 * err
        if e2 >= dy:
            err += dy
            x0 += sx
        if e2 <= dx:
            err += dx
            y0 += sy


def fill_quad(mask: np.ndarray, pts, value=255) -> np.ndarray:
    """cv2.drawContours(mask, [pts], -1, value, thickness=FILLED) for one integer polygon:
    the polygon's edges drawn as 8-connected lines, plus an even-odd scanline fill of each row
    y between the edges' crossings (fixed point 16.16 as OpenCV's FillEdgeCollection: an edge
    from its upper vertex with x step trunc(dx * 65536 / dy); pixels ceil(x_left)..floor(x_right);
    an edge covers rows y0 <= y < y1)."""
    p = np.asarray(pts, dtype=np.int64).reshape(-1, 2)
    n = len(p)
    if n == 0:
        return mask
    for i in range(n):
        _line8(mask, p[i - 1], p[i], value)
    edges = []
    for i in range(n):
        (xa, ya), (xb, yb) = p[i - 1], p[i]
        if ya == yb:
            continue
        if ya > yb:
            xa, ya, xb, yb = xb, yb, xa, ya
        num = (int(xb) - int(xa)) << 16
        den = int(yb - ya)
        step = abs(num) // den * (1 if num >= 0 else -1)  # C integer division truncates
        edges.append((int(ya), int(yb), int(xa) << 16, step))
    if len(edges) < 2:
        return mask
    H, W = mask.shape[:2]
    y_lo = max(min(e[0] for e in edges), 0)
    y_hi = min(max(e[1] for e in edges), H)
    for y in range(y_lo, y_hi):
        xs = sorted(x0 + (y - ya) * st for ya, yb, x0, st in edges if ya <= y < yb)
        for k in range(0, len(xs) - 1, 2):
            xl = (xs[k] + 0xFFFF) >> 16
            xr = xs[k + 1] >> 16
            xl, xr = max(xl, 0), min(xr, W - 1)
            if xl <= xr:
                mask[y, xl:xr + 1] = value
    return mask


def _trace_outer(img: np.ndarray, i: int, j: int) -> List[Tuple[int, int]]:
    """Suzuki-Abe outer border following from the component's first raster pixel (i, j)
    (its west neighbour is background).  img is zero-padded; returns (x, y) points."""
    def nz(d, ci, cj):
        di, dj = _DIRS[d]
        return img[ci + di, cj + dj] != 0

    # 3.1: clockwise from the west neighbour (direction 4) for the first foreground pixel
    start = 4
    d1 = None
    for k in range(8):
        d = (start - k) % 8
        if nz(d, i, j):
            d1 = d
            break
    pts = [(j, i)]
    if d1 is None:
        return pts
    i1, j1 = i + _DIRS[d1][0], j + _DIRS[d1][1]
    i3, j3 = i, j
    d2 = d1  # direction from (i3, j3) to (i2, j2)
    while True:
        # 3.3: counter-clockwise from the element after (i2, j2)
        d4 = None
        for k in range(1, 9):
            d = (d2 + k) % 8
            if nz(d, i3, j3):
                d4 = d
                break
        i4, j4 = i3 + _DIRS[d4][0], j3 + _DIRS[d4][1]
        if i4 == i and j4 == j and i3 == i1 and j3 == j1:
            return pts
        # (i2, j2) <- (i3, j3); the direction from (i4, j4) back to (i3, j3)
        d2 = (d4 + 4) % 8
        i3, j3 = i4, j4
        if (j3, i3) == pts[0] and len(pts) > 1 and i3 == i and j3 == j:
            pass
        pts.append((j3, i3))


def contour_area(pts) -> float:
    """cv2.contourArea (unoriented shoelace area of the point chain)."""
    if len(pts) < 3:
        return 0.0
    a = np.asarray(pts, dtype=np.float64)
    x, y = a[:, 0], a[:, 1]
    return float(abs(np.dot(x, np.roll(y, -1)) - np.dot(np.roll(x, -1), y)) / 2.0)


def bounding_rect(pts) -> Tuple[int, int, int, int]:
    a = np.asarray(pts, dtype=np.int64)
    x0, y0 = a.min(0)
    x1, y1 = a.max(0)
    return int(x0), int(y0), int(x1 - x0 + 1), int(y1 - y0 + 1)


def external_contours(binary: np.ndarray) -> List[List[Tuple[int, int]]]:
    """Outer borders of the 8-connected foreground components that are not inside another
    component's hole (RETR_EXTERNAL), in raster order of their first pixel; each contour is a
    list of (x, y) boundary pixel centres (the image outside its frame counts as background)."""
    from scipy import ndimage
    fg = np.asarray(binary) != 0
    H, W = fg.shape
    pad = np.zeros((H + 2, W + 2), np.uint8)
    pad[1:-1, 1:-1] = fg
    lab, n = ndimage.label(pad, structure=np.ones((3, 3), bool))
    if n == 0:
        return []
    # background 4-connected to the frame: components touching it are external
    bg, _ = ndimage.label(pad == 0, structure=ndimage.generate_binary_structure(2, 1))
    outer = bg == bg[0, 0]
    touch = ndimage.binary_dilation(outer, structure=ndimage.generate_binary_structure(2, 1)) & (lab > 0)
    external = set(np.unique(lab[touch]).tolist()) - {0}
    # first pixel (raster order) of each component
    flat = lab.ravel()
    order = np.flatnonzero(flat)
    first = {}
    for idx in order[np.unique(flat[order], return_index=True)[1]]:
        first[int(flat[idx])] = idx
    out = []
    for lbl in sorted(external, key=lambda l: first[l]):
        i, j = divmod(int(first[lbl]), W + 2)
        comp = (lab == lbl).astype(np.uint8)
        pts = _trace_outer(comp, i, j)
        out.append([(x - 1, y - 1) for x, y in pts])
    return out


def largest_external_contour(binary: np.ndarray):
    """(area, (x, y, w, h)) of the external contour of largest cv2.contourArea (first on ties),
    or None if there is no foreground."""
    best = None
    for c in external_contours(binary):
        a = contour_area(c)
        if best is None or a > best[0]:
            best = (a, bounding_rect(c))
    return best
