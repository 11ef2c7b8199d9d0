"""Torch-tensor front end of the C-ABI: argument checking, pointers, streams, workspaces.

PyTorch is plumbing here (device memory, the current HIP stream, torch.distributed);
every computation is a libunet_hip.so kernel.  Tensors must be contiguous float32 on a
HIP device; ops run asynchronously on torch's current stream.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, replace
from typing import Optional, Tuple

import torch

from . import _lib as L
from ._lib import UnetView

Tensor = torch.Tensor


def _ptr(t: Optional[Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class DeviceEvent:
    """Cross-stream ordering event of one device (unet_event_create: no timing, device-scope
    release only).  wait(waiter, producer) = waiter.wait_stream(producer) without the default
    event's system-scope fence."""

    def __init__(self):
        h = ctypes.c_void_p()
        L.call("unet_event_create", ctypes.byref(h))
        self._h = h

    def wait(self, waiter, producer):
        L.call("unet_stream_wait_stream", ctypes.c_void_p(waiter.cuda_stream), ctypes.c_void_p(producer.cuda_stream),
               self._h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.load().unet_event_destroy(h)
            except Exception:
                pass
            self._h = None


def _check(t: Tensor, name: str, numel: Optional[int] = None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a device (HIP) tensor; there is no CPU path")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name}: expected {numel} elements, got {t.numel()}")


class _Workspace:
    """Per-(device, stream) growable scratch buffer (stream order makes reuse safe)."""

    def __init__(self):
        self._bufs = {}

    def get(self, nbytes: int, device) -> Tensor:
        key = (torch.device(device).index, torch.cuda.current_stream(device).cuda_stream)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            nb = max(int(nbytes * 1.25), 1 << 20)
            buf = torch.empty(nb, dtype=torch.uint8, device=device)
            self._bufs[key] = buf
        return buf


WORKSPACE = _Workspace()


PEAK_FP32_FLOPS = 157.3e12  # MI355X dense FP32 (matrix = vector rate), MI355X_MICROARCH.md
PEAK_HBM_BYTES = 8.0e12


class KernelTimer:
    """Brackets selected C-ABI ops with HIP events on the stream they are launched on
    (torch's current stream) and accumulates their algorithmic flops / bytes, so a bench
    can report achieved throughput of one kernel over a timed region.  Each record also carries
    the op's route (which kernels the call launches, e.g. the 1024-channel data gradients' dz
    pass + plain GEMM), so PMC kernel counts can be matched to the same launch set."""

    def __init__(self, names=None):
        self.names = None if names is None else set(names)  # None: every op
        self.records = []  # (name, route, flops, bytes, start_event, end_event)

    def summary(self):
        """Per op: launches, ms, flops, bytes, t_roof_ms = sum over launches of
        max(flops / peak_fp32, bytes / peak_hbm) (each launch against its own bound), and the
        same per route."""
        torch.cuda.synchronize()
        out = {}
        for name, route, fl, nb, e0, e1 in self.records:
            ms = e0.elapsed_time(e1)
            tr = max(fl / PEAK_FP32_FLOPS, nb / PEAK_HBM_BYTES) * 1e3
            for d in (out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "t_roof_ms": 0.0,
                                            "hbm_bound_launches": 0, "routes": {}}),):
                for dd in (d, d["routes"].setdefault(route, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0,
                                                              "t_roof_ms": 0.0})):
                    dd["launches"] += 1
                    dd["ms"] += ms
                    dd["flops"] += fl
                    dd["bytes"] += nb
                    dd["t_roof_ms"] += tr
                if nb / PEAK_HBM_BYTES > fl / PEAK_FP32_FLOPS:
                    d["hbm_bound_launches"] += 1
        return out


TIMER: Optional[KernelTimer] = None


def _call(name: str, work, *args, route: str = "main"):
    """L.call, bracketed by HIP events when TIMER selects `name`; work = (flops, bytes)."""
    t = TIMER
    if t is None or (t.names is not None and name not in t.names):
        L.call(name, *args)
        return
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    L.call(name, *args)
    e1.record()
    t.records.append((name, route, float(work[0]), float(work[1]), e0, e1))


def _ws(nbytes: int, device):
    if nbytes <= 0:
        return None, 0
    buf = WORKSPACE.get(nbytes, device)
    return _ptr(buf), buf.numel()


def _planes(t: Optional[Tensor], numel: int, what: str):
    if t is not None and (t.dtype != torch.int16 or t.numel() < 3 * numel or not t.is_cuda):
        raise ValueError(f"{what}: split-precision planes must be 3 x {numel} int16 on the device")
    return t


# ---------------------------------------------------------------------------- views ---
@dataclass
class View:
    """Python side of `unet_view`: how a layer reads its logical input (see unet_hip.h)."""

    mode: int
    src0: Tensor
    c0: int
    scale0: Optional[Tensor] = None
    shift0: Optional[Tensor] = None
    src1: Optional[Tensor] = None
    c1: int = 0
    scale1: Optional[Tensor] = None
    shift1: Optional[Tensor] = None
    drop_rate: float = 0.0
    drop_seed: int = 0

    @property
    def channels(self) -> int:
        return self.c0 + (self.c1 if self.mode == L.VIEW_CONCAT else 0)

    @staticmethod
    def plain(x: Tensor) -> "View":
        return View(L.VIEW_PLAIN, x, x.shape[-1])

    @staticmethod
    def bnrelu(z: Tensor, scale: Tensor, shift: Tensor) -> "View":
        return View(L.VIEW_BNRELU, z, z.shape[-1], scale, shift)

    @staticmethod
    def pool_bnrelu(z: Tensor, scale: Tensor, shift: Tensor) -> "View":
        return View(L.VIEW_POOL_BNRELU, z, z.shape[-1], scale, shift)

    @staticmethod
    def concat(up: Tensor, skip_z: Tensor, scale: Tensor, shift: Tensor) -> "View":
        return View(L.VIEW_CONCAT, up, up.shape[-1], None, None, skip_z, skip_z.shape[-1], scale, shift)

    def src_bytes(self, n: int, h: int, w: int) -> float:
        """Algorithmic bytes of one pass over the view's sources at logical size (n, h, w)."""
        px = float(n * h * w)
        if self.mode == L.VIEW_POOL_BNRELU:
            return 16.0 * px * self.c0
        return 4.0 * px * self.channels

    def dropout(self, rate: float, seed: int) -> "View":
        return replace(self, drop_rate=float(rate), drop_seed=int(seed) & 0xFFFFFFFFFFFFFFFF)

    def batch(self, sl: slice) -> "View":
        """The view of images sl of the batch (sources sliced along dim 0).  Not for dropout
        views: the mask is drawn from the element's linear index in the whole batch."""
        if self.drop_rate > 0.0:
            raise ValueError("batch slices of a dropout view would draw a different mask")
        return replace(self, src0=self.src0[sl], src1=self.src1[sl] if self.src1 is not None else None)

    def c_struct(self) -> UnetView:
        for name in ("src0", "scale0", "shift0", "src1", "scale1", "shift1"):
            t = getattr(self, name)
            if t is not None:
                _check(t, f"view.{name}")
        v = UnetView()
        v.mode = self.mode
        v.c0 = self.c0
        v.c1 = self.c1 if self.mode == L.VIEW_CONCAT else 0
        v.src0 = self.src0.data_ptr()
        v.scale0 = self.scale0.data_ptr() if self.scale0 is not None else None
        v.shift0 = self.shift0.data_ptr() if self.shift0 is not None else None
        v.src1 = self.src1.data_ptr() if self.src1 is not None else None
        v.scale1 = self.scale1.data_ptr() if self.scale1 is not None else None
        v.shift1 = self.shift1.data_ptr() if self.shift1 is not None else None
        v.drop_rate = self.drop_rate
        v.drop_seed = self.drop_seed
        return v


def view_materialize(x: View, n: int, h: int, w: int, out: Tensor) -> Tensor:
    _check(out, "out", n * h * w * x.channels)
    vs = x.c_struct()
    _call("unet_view_materialize", (0.0, x.src_bytes(n, h, w) + 4.0 * out.numel()), ctypes.byref(vs), n, h, w,
          _ptr(out), _stream())
    return out


# --------------------------------------------------------------- SeparableConv2D ---
def copy_strided(src: Tensor, rows: int, cols: int, src_ld: int, dst: Tensor, dst_ld: int) -> None:
    """dst[r * dst_ld + c] = src[r * src_ld + c] (r < rows, c < cols): channel padding / slicing."""
    _check(src, "src")
    _check(dst, "dst")
    if rows and (src.numel() < (rows - 1) * src_ld + cols or dst.numel() < (rows - 1) * dst_ld + cols):
        raise ValueError("copy_strided: tensors too small for rows x cols at the given strides")
    _call("unet_copy_strided", (0.0, 8.0 * rows * cols), _ptr(src), rows, cols, src_ld, _ptr(dst), dst_ld, _stream())


def dwconv3x3_fwd(x: View, n: int, h: int, w: int, dk: Tensor, out: Tensor) -> Tensor:
    C = x.channels
    _check(dk, "depthwise_kernel", 9 * C)
    _check(out, "out", n * h * w * C)
    vs = x.c_struct()
    _call("unet_dwconv3x3_fwd", (18.0 * n * h * w * C, x.src_bytes(n, h, w) + 4.0 * (n * h * w * C + 9 * C)),
          ctypes.byref(vs), n, h, w, _ptr(dk), _ptr(out), _stream())
    return out


def dwconv3x3_bwd_data(x: View, n, h, w, dk: Tensor, dy: Tensor, dx0: Tensor, dx1: Optional[Tensor] = None):
    C = x.channels
    _check(dk, "depthwise_kernel", 9 * C)
    _check(dy, "dy", n * h * w * C)
    _check(dx0, "dx0")
    if dx1 is not None:
        _check(dx1, "dx1")
    vs = x.c_struct()
    m = n * h * w
    # read dy, write dx; the pool route also reads the 2x2 sources and read-modify-writes dx0
    nb = 8.0 * m * C + (3.0 * x.src_bytes(n, h, w) if x.mode == L.VIEW_POOL_BNRELU else 0.0)
    _call("unet_dwconv3x3_bwd_data", (18.0 * m * C, nb), ctypes.byref(vs), n, h, w, _ptr(dk), _ptr(dy), _ptr(dx0),
          _ptr(dx1), _stream())


def dwconv3x3_bwd_data_bnstats_slabs(x: View, n, h, w) -> int:
    """Slab count of dwconv3x3_bwd_data_bnstats's BatchNorm partials (0: no fused path)."""
    vs = x.c_struct()
    return L.query("unet_dwconv3x3_bwd_data_bnstats_slabs", ctypes.byref(vs), n, h, w)


def dwconv3x3_bwd_data_bnstats(x: View, n, h, w, dk: Tensor, dy: Tensor, dx0: Tensor, mean, rstd,
                               partials: Tensor):
    """POOL view: dwconv3x3_bwd_data that also emits the pooled block's BN-backward partials."""
    C = x.channels
    S = dwconv3x3_bwd_data_bnstats_slabs(x, n, h, w)
    _check(dk, "depthwise_kernel", 9 * C)
    _check(dy, "dy", n * h * w * C)
    _check(dx0, "dx0")
    _check(partials, "bn_partials", bn_stats_partials_numel(S, C))
    vs = x.c_struct()
    m = n * h * w
    # read dy, write dx; pool: the 2x2 sources and the read-modify-write of dx0; BN+ReLU: z once
    nb = 8.0 * m * C + (3.0 * x.src_bytes(n, h, w) if x.mode == L.VIEW_POOL_BNRELU else 4.0 * m * C) + 4.0 * S * 2 * C
    _call("unet_dwconv3x3_bwd_data_bnstats", (18.0 * m * C, nb), ctypes.byref(vs), n, h, w, _ptr(dk), _ptr(dy),
          _ptr(dx0), _ptr(mean), _ptr(rstd), _ptr(partials), _stream())


def dwconv3x3_bwd_data_bnstats_dwf(x: View, n, h, w, dk: Tensor, dy: Tensor, dx0: Tensor, mean, rstd,
                                   partials: Tensor, dw_partials: Tensor):
    """BNRELU view (no dropout): dwconv3x3_bwd_data_bnstats that also writes the depthwise filter
    gradient's per-tile slabs ([S][9][C]; sum them with reduce_slabs)."""
    C = x.channels
    S = dwconv3x3_bwd_data_bnstats_slabs(x, n, h, w)
    _check(dk, "depthwise_kernel", 9 * C)
    _check(dy, "dy", n * h * w * C)
    _check(dx0, "dx0")
    _check(partials, "bn_partials", bn_stats_partials_numel(S, C))
    _check(dw_partials, "dw_partials", S * 9 * C)
    vs = x.c_struct()
    m = n * h * w
    nb = 12.0 * m * C + 4.0 * S * 2 * C + 4.0 * S * 9 * C
    _call("unet_dwconv3x3_bwd_data_bnstats_dwf", (36.0 * m * C, nb), ctypes.byref(vs), n, h, w, _ptr(dk), _ptr(dy),
          _ptr(dx0), _ptr(mean), _ptr(rstd), _ptr(partials), _ptr(dw_partials), _stream())


def reduce_slabs(slabs: Tensor, S: int, length: int, out: Tensor):
    """out = sum of S slabs of `length` floats, fixed order (slabs is scratch: overwritten)."""
    _check(slabs, "slabs", S * length)
    _check(out, "out", length)
    _call("unet_reduce_slabs", (0.0, 4.0 * S * length), _ptr(slabs), S, length, _ptr(out), _stream())


def dwconv3x3_bwd_filter(x: View, n, h, w, dy: Tensor, ddk: Tensor):
    C = x.channels
    _check(dy, "dy", n * h * w * C)
    _check(ddk, "d_depthwise_kernel", 9 * C)
    ws, wsb = _ws(L.query("unet_dwconv3x3_bwd_filter_workspace", n, h, w, C), dy.device)
    vs = x.c_struct()
    _call("unet_dwconv3x3_bwd_filter", (18.0 * n * h * w * C, x.src_bytes(n, h, w) + 4.0 * n * h * w * C),
          ctypes.byref(vs), n, h, w, _ptr(dy), _ptr(ddk), ws, wsb, _stream())


def bn_partials_numel(m: int, c: int) -> int:
    """Floats of a forward BN partials buffer; allocate it zeroed (bn_finalize's counters)."""
    return L.query("unet_bn_partials_size", m, c) // 4


def pointwise_fwd(y: Tensor, m: int, cin: int, cout: int, pk: Tensor, z: Tensor, partials: Optional[Tensor] = None,
                  pkx: Optional[Tensor] = None):
    """pkx: pk's split-precision planes ([3][cout][cin], split_x3): the bf16x6 GEMM where cin % 32 == 0."""
    _check(y, "y", m * cin)
    _check(pk, "pointwise_kernel", cin * cout)
    _check(z, "z", m * cout)
    if partials is not None:
        _check(partials, "bn_partials", bn_partials_numel(m, cout))
    work = (2.0 * m * cin * cout, 4.0 * (m * cin + m * cout + cin * cout))
    if _planes(pkx, cin * cout, "pointwise_fwd") is not None:
        _call("unet_pointwise_fwd_x3", work, _ptr(y), m, cin, cout, _ptr(pk), _ptr(pkx), _ptr(z), _ptr(partials),
              _stream())
        return
    _call("unet_pointwise_fwd", work, _ptr(y), m, cin, cout, _ptr(pk), _ptr(z), _ptr(partials), _stream())


def pointwise_bwd_data(dz: Tensor, m, cin, cout, pk: Tensor, dy: Tensor):
    _check(dz, "dz", m * cout)
    _check(pk, "pointwise_kernel", cin * cout)
    _check(dy, "dy", m * cin)
    _call("unet_pointwise_bwd_data", (2.0 * m * cin * cout, 4.0 * (m * cin + m * cout + cin * cout)), _ptr(dz), m,
          cin, cout, _ptr(pk), _ptr(dy), _stream())


def pointwise_bwd_filter(y: Tensor, dz: Tensor, m, cin, cout, dpk: Tensor):
    _check(y, "y", m * cin)
    _check(dz, "dz", m * cout)
    _check(dpk, "d_pointwise_kernel", cin * cout)
    ws, wsb = _ws(L.query("unet_pointwise_bwd_filter_workspace", m, cin, cout), y.device)
    _call("unet_pointwise_bwd_filter", (2.0 * m * cin * cout, 4.0 * (m * cin + m * cout + cin * cout)), _ptr(y),
          _ptr(dz), m, cin, cout, _ptr(dpk), ws, wsb, _stream())


SEPCONV_AUTO, SEPCONV_TILE, SEPCONV_RK, SEPCONV_RK1 = 0, 1, 2, 3


def sepconv_set_schedule(schedule: int) -> int:
    """Kernel schedule of sepconv_fwd (see unet_sepconv_set_schedule); returns the previous one."""
    r = L.load().unet_sepconv_set_schedule(int(schedule))
    if r < 0:
        raise ValueError(f"bad sepconv schedule {schedule}")
    return r


def sepconv_supported(x: View, n: int, h: int, w: int, cout: int) -> bool:
    vs = x.c_struct()
    return bool(L.load().unet_sepconv_fwd_supported(ctypes.byref(vs), n, h, w, cout))


def split_x3(src: Tensor, segs, dst: Tensor, keep: bool = False):
    """bf16 x 3 split-precision planes of several weight matrices in one launch: segs = [(source
    offset, rows, cols, destination offset)] in elements of src (float32) / dst (int16 holding
    bf16 bits); each segment becomes planes [3][cols][rows] at its destination offset
    (keep=True: [3][rows][cols], the source layout -- unet_split_x3_keep).  Segments of five
    (..., keep flag) mix both layouts in one launch (unet_split_x3_mixed)."""
    if src.dtype != torch.float32 or dst.dtype != torch.int16:
        raise TypeError("split_x3: float32 source, int16 (bf16 bits) destination")
    mixed = len(segs) > 0 and len(segs[0]) == 5
    if len(segs) > L.SPLIT_MAX_SEGS or any(len(sg) != (5 if mixed else 4) for sg in segs):
        raise ValueError("split_x3: bad segment list")
    flat = [int(v) for seg in segs for v in seg]
    for so, r, c, do, *_ in segs:
        if so + r * c > src.numel() or do + 3 * r * c > dst.numel():
            raise ValueError("split_x3: segment out of range")
    arr = (ctypes.c_int64 * len(flat))(*flat)
    name = "unet_split_x3_mixed" if mixed else ("unet_split_x3_keep" if keep else "unet_split_x3")
    _call(name, (0.0, sum(10.0 * sg[1] * sg[2] for sg in segs)), _ptr(src), arr, len(segs), _ptr(dst), _stream())


def sepconv_fwd(x: View, n: int, h: int, w: int, dk: Tensor, cout: int, pk: Tensor, y: Optional[Tensor],
                z: Tensor, partials: Optional[Tensor] = None, zsel: Optional[Tensor] = None,
                gamma: Optional[Tensor] = None, pkx: Optional[Tensor] = None):
    """Fused depthwise 3x3 + pointwise 1x1 (+ BN partials); y (depthwise output) optional; zsel
    (optional, (n, h/2, w/2, cout)): the 2x2 max-pool selection of z for the next stage (see
    unet_pool_select; gamma = the block's BN gamma, None without BatchNorm); pkx (optional): pk's
    split-precision planes from split_x3 (the kernel's bf16x6 MFMA variant where it exists)."""
    C = x.channels
    m = n * h * w
    _check(dk, "depthwise_kernel", 9 * C)
    _check(pk, "pointwise_kernel", C * cout)
    _check(z, "z", m * cout)
    if y is not None:
        _check(y, "y", m * C)
    if partials is not None:
        _check(partials, "bn_partials", bn_partials_numel(m, cout))
    if zsel is not None:
        _check(zsel, "z_pool_sel", m * cout // 4)
    if gamma is not None:
        _check(gamma, "gamma", cout)
    if pkx is not None and (pkx.dtype != torch.int16 or pkx.numel() < 3 * C * cout or not pkx.is_cuda):
        raise ValueError("sepconv_fwd: pkx must be the int16 split planes of pk (3 * Cin * Cout)")
    vs = x.c_struct()
    nb = x.src_bytes(n, h, w) + 4.0 * (m * cout + C * cout + 9 * C) + (4.0 * m * C if y is not None else 0.0) + \
        (1.0 * m * cout if zsel is not None else 0.0)
    _call("unet_sepconv_fwd", (2.0 * m * C * cout + 18.0 * m * C, nb),
          ctypes.byref(vs), n, h, w, _ptr(dk), cout, _ptr(pk), _ptr(pkx), _ptr(y), _ptr(z), _ptr(partials),
          _ptr(zsel), _ptr(gamma), _stream())


def pool_select(z: Tensor, n: int, h: int, w: int, c: int, gamma: Optional[Tensor], out: Tensor):
    """out (n, h/2, w/2, c): per 2x2 window the raw z the max-pool of relu(bn(z)) selects."""
    _check(z, "z", n * h * w * c)
    _check(out, "out", n * h * w * c // 4)
    if gamma is not None:
        _check(gamma, "gamma", c)
    _call("unet_pool_select", (0.0, 5.0 * n * h * w * c), _ptr(z), n, h, w, c, _ptr(gamma), _ptr(out), _stream())


def sepconv_bwd_filter_supported(x: View, n: int, h: int, w: int, cout: int) -> bool:
    vs = x.c_struct()
    return bool(L.load().unet_sepconv_bwd_filter_supported(ctypes.byref(vs), n, h, w, cout))


def sepconv_bwd_fused(x: View, n: int, h: int, w: int, dk: Tensor, pk: Tensor, da: Optional[Tensor], z: Tensor,
                      scale: Tensor, shift: Tensor, coef: Tensor, cout: int, dy: Tensor, ddk: Tensor, dpk: Tensor,
                      da_rank1: Optional[Tuple[Tensor, Tensor]] = None):
    """A 64-output block's BN + ReLU backward, pointwise data gradient and both weight gradients
    in one pass (dz never stored): dy out, d_depthwise / d_pointwise kernels overwritten.
    da_rank1 = (dlogit (m,), head kernel (cout,)) instead of da: the binary head's rank-one
    gradient, formed on load."""
    C = x.channels
    m = n * h * w
    _check(dk, "depthwise_kernel", 9 * C)
    _check(pk, "pointwise_kernel", C * cout)
    if (da is None) == (da_rank1 is None):
        raise ValueError("sepconv_bwd_fused: give da or da_rank1")
    if da is not None:
        _check(da, "da", m * cout)
        da_bytes = 4.0 * m * cout
    else:
        _check(da_rank1[0], "da_dlogit", m)
        _check(da_rank1[1], "da_kernel", cout)
        da_bytes = 4.0 * m
    _check(z, "z", m * cout)
    _check(coef, "coef", 3 * cout)
    _check(dy, "dy", m * C)
    _check(ddk, "d_depthwise_kernel", 9 * C)
    _check(dpk, "d_pointwise_kernel", C * cout)
    ws, wsb = _ws(L.query("unet_sepconv_bwd_filter_workspace", n, h, w, C, cout), dy.device)
    vs = x.c_struct()
    _call("unet_sepconv_bwd_fused", (4.0 * m * C * cout + 36.0 * m * C,
                                     x.src_bytes(n, h, w) + 4.0 * (m * C + m * cout) + da_bytes),
          ctypes.byref(vs), n, h, w, _ptr(dk), _ptr(pk), _ptr(da), _ptr(da_rank1[0] if da_rank1 else None),
          _ptr(da_rank1[1] if da_rank1 else None), _ptr(z), _ptr(scale), _ptr(shift), _ptr(coef), cout,
          _ptr(dy), _ptr(ddk), _ptr(dpk), ws, wsb, _stream())


def sepconv_bwd_filter(x: View, n: int, h: int, w: int, dk: Tensor, dy: Tensor, dz: Tensor, cout: int,
                       ddk: Tensor, dpk: Tensor):
    """Depthwise and pointwise kernel gradients in one pass, y recomputed from the view x."""
    C = x.channels
    m = n * h * w
    _check(dk, "depthwise_kernel", 9 * C)
    _check(dy, "dy", m * C)
    _check(dz, "dz", m * cout)
    _check(ddk, "d_depthwise_kernel", 9 * C)
    _check(dpk, "d_pointwise_kernel", C * cout)
    ws, wsb = _ws(L.query("unet_sepconv_bwd_filter_workspace", n, h, w, C, cout), dy.device)
    vs = x.c_struct()
    _call("unet_sepconv_bwd_filter", (2.0 * m * C * cout + 36.0 * m * C,
                                      x.src_bytes(n, h, w) + 4.0 * (m * C + m * cout)),
          ctypes.byref(vs), n, h, w, _ptr(dk), _ptr(dy), _ptr(dz), cout, _ptr(ddk), _ptr(dpk), ws, wsb, _stream())


# ------------------------------------------------------------------ BatchNorm ---
def bn_finalize(partials: Tensor, m: int, c: int, gamma, beta, eps, momentum, moving_mean, moving_var,
                update_moving: bool, mean, rstd, scale, shift):
    _call("unet_bn_finalize", (0.0, 8.0 * bn_partials_numel(m, c) / 2), _ptr(partials), m, c, _ptr(gamma), _ptr(beta), float(eps), float(momentum),
           _ptr(moving_mean), _ptr(moving_var), int(bool(update_moving)), _ptr(mean), _ptr(rstd), _ptr(scale),
           _ptr(shift), _stream())


def bn_moments(partials: Tensor, m: int, c: int, out: Tensor):
    """SyncBN: this replica's record (count, mean[c], M2[c]) as 1 + 2c float64 (unet_bn_moments)."""
    _check(partials, "bn_partials", bn_partials_numel(m, c))
    if out.dtype != torch.float64 or out.numel() < 1 + 2 * c or not out.is_cuda:
        raise ValueError("bn_moments: out must be a float64 device tensor of 1 + 2c elements")
    _call("unet_bn_moments", (0.0, 8.0 * bn_partials_numel(m, c) / 2), _ptr(partials), m, c, _ptr(out), _stream())


def bn_finalize_moments(records: Tensor, world: int, c: int, gamma, beta, eps, momentum, moving_mean, moving_var,
                        update_moving: bool, mean, rstd, scale, shift):
    """SyncBN: the gathered records [world][1 + 2c] combined in rank order, then finalized."""
    if records.dtype != torch.float64 or records.numel() < world * (1 + 2 * c) or not records.is_cuda:
        raise ValueError("bn_finalize_moments: records must be float64 [world][1 + 2c] on the device")
    _call("unet_bn_finalize_moments", (0.0, 8.0 * world * (1 + 2 * c)), _ptr(records), world, c, _ptr(gamma),
          _ptr(beta), float(eps), float(momentum), _ptr(moving_mean), _ptr(moving_var), int(bool(update_moving)),
          _ptr(mean), _ptr(rstd), _ptr(scale), _ptr(shift), _stream())


def bn_bwd_coef(sums: Tensor, m: int, c: int, use_bn: bool, mean, rstd, coef: Tensor):
    """SyncBN backward: coef (3c) from the all-reduced [sum g | sum g*xhat] (2c) over m pixels."""
    _check(sums, "sums", 2 * c)
    _check(coef, "coef", 3 * c)
    _call("unet_bn_bwd_coef", (0.0, 24.0 * c), _ptr(sums), m, c, int(bool(use_bn)), _ptr(mean), _ptr(rstd),
          _ptr(coef), _stream())


def bn_infer_params(gamma, beta, moving_mean, moving_var, c: int, eps, scale: Tensor, shift: Tensor):
    _call("unet_bn_infer_params", (0.0, 24.0 * c), _ptr(gamma), _ptr(beta), _ptr(moving_mean), _ptr(moving_var), c, float(eps),
           _ptr(scale), _ptr(shift), _stream())


def bn_relu_bwd(da: Tensor, z: Tensor, m: int, c: int, mean, rstd, scale, shift, use_bn: bool, drop_rate: float,
                drop_seed: int, dgamma, dbeta, dz: Tensor):
    _check(da, "da", m * c)
    _check(z, "z", m * c)
    _check(dz, "dz", m * c)
    ws, wsb = _ws(L.query("unet_bn_relu_bwd_workspace", m, c), z.device)
    _call("unet_bn_relu_bwd", (12.0 * m * c, 12.0 * m * c), _ptr(da), _ptr(z), m, c, _ptr(mean), _ptr(rstd), _ptr(scale), _ptr(shift),
           int(bool(use_bn)), float(drop_rate), int(drop_seed) & 0xFFFFFFFFFFFFFFFF, _ptr(dgamma), _ptr(dbeta),
           _ptr(dz), ws, wsb, _stream())


def bn_relu_bwd_stats(da: Tensor, z: Tensor, m: int, c: int, mean, rstd, scale, shift, use_bn: bool,
                      drop_rate: float, drop_seed: int, dgamma, dbeta, coef: Tensor):
    """Statistics half of bn_relu_bwd: dgamma / dbeta and coef (3c) for pointwise_bwd_data_bnrelu."""
    _check(da, "da", m * c)
    _check(z, "z", m * c)
    _check(coef, "coef", 3 * c)
    ws, wsb = _ws(L.query("unet_bn_relu_bwd_workspace", m, c), z.device)
    _call("unet_bn_relu_bwd_stats", (8.0 * m * c, 8.0 * m * c), _ptr(da), _ptr(z), m, c, _ptr(mean), _ptr(rstd),
          _ptr(scale), _ptr(shift), int(bool(use_bn)), float(drop_rate), int(drop_seed) & 0xFFFFFFFFFFFFFFFF,
          _ptr(dgamma), _ptr(dbeta), _ptr(coef), ws, wsb, _stream())


def bn_stats_partials_numel(S: int, c: int) -> int:
    """Floats of a producer-side BN partials buffer of S slabs (slabs + finish scratch + counters).

    Allocate it zeroed (torch.zeros): bn_relu_bwd_stats_finish needs its counters zero on entry.
    """
    return L.query("unet_bn_stats_partials_size", S, c) // 4


def bn_relu_bwd_stats_finish(partials: Tensor, S: int, m: int, c: int, mean, rstd, use_bn: bool, dgamma, dbeta,
                             coef: Tensor):
    """bn_relu_bwd_stats's outputs from producer-side partial slabs ([S][2][c])."""
    _check(partials, "bn_partials", bn_stats_partials_numel(S, c))
    _check(coef, "coef", 3 * c)
    _call("unet_bn_relu_bwd_stats_finish", (2.0 * S * c, 8.0 * S * c), _ptr(partials), S, m, c, _ptr(mean),
          _ptr(rstd), int(bool(use_bn)), _ptr(dgamma), _ptr(dbeta), _ptr(coef), _stream())


def pointwise_bwd_data_bnrelu(da: Tensor, z: Tensor, m: int, cin: int, cout: int, pk: Tensor, scale: Tensor,
                              shift: Tensor, coef: Tensor, drop_rate: float, drop_seed: int, dy: Tensor,
                              dz: Optional[Tensor], pkd: Optional[Tensor] = None):
    """dy = dz . pk^T with dz (BN + ReLU + dropout backward) formed on load; optionally stores dz.
    pkd: pk's split-precision planes in its own layout (split_x3(keep=True)): the bf16x6 GEMM
    (unet_pointwise_bwd_data_bnrelu_x3) where cout % 32 == 0."""
    _check(da, "da", m * cout)
    _check(z, "z", m * cout)
    _check(pk, "pointwise_kernel", cin * cout)
    _check(coef, "coef", 3 * cout)
    _check(dy, "dy", m * cin)
    if dz is not None:
        _check(dz, "dz", m * cout)
    # (measurement label only) the library forms dz in a streaming pass and runs the plain GEMM
    # when either side has >= 1024 channels (gemm.hip, unet_pointwise_bwd_data_bnrelu)
    route = "dz_pass+gemm" if dz is not None and (cin >= 1024 or cout >= 1024) else "gemm_bnbwd"
    work = (2.0 * m * cin * cout, 4.0 * (2 * m * cout + m * cin + cin * cout) + (4.0 * m * cout if dz is not None else 0))
    if pkd is not None:
        if pkd.dtype != torch.int16 or pkd.numel() < 3 * cin * cout or not pkd.is_cuda:
            raise ValueError("pointwise_bwd_data_bnrelu: pkd must be 3 x cin x cout int16 planes on the device")
        _call("unet_pointwise_bwd_data_bnrelu_x3", work, _ptr(da), _ptr(z), m, cin, cout, _ptr(pk), _ptr(pkd),
              _ptr(scale), _ptr(shift), _ptr(coef), float(drop_rate), int(drop_seed) & 0xFFFFFFFFFFFFFFFF, _ptr(dy),
              _ptr(dz), _stream(), route=route + ("_x6" if cout % 32 == 0 else ""))
        return
    _call("unet_pointwise_bwd_data_bnrelu", work,
          _ptr(da), _ptr(z), m, cin, cout, _ptr(pk), _ptr(scale), _ptr(shift), _ptr(coef), float(drop_rate),
          int(drop_seed) & 0xFFFFFFFFFFFFFFFF, _ptr(dy), _ptr(dz), _stream(), route=route)


def pointwise_bwd_data_bnrelu_wgrad(da: Tensor, z: Tensor, m: int, cin: int, cout: int, pk: Tensor, scale: Tensor,
                                    shift: Tensor, coef: Tensor, y: Tensor, dy: Tensor, dpk: Tensor):
    """pointwise_bwd_data_bnrelu (no dropout) for cin == 4 that also writes the pointwise weight
    gradient dpk[ci][co] = sum_m y[m, ci] dz[m, co] from the dz it forms (dz is not stored)."""
    _check(da, "da", m * cout)
    _check(z, "z", m * cout)
    _check(pk, "pointwise_kernel", cin * cout)
    _check(coef, "coef", 3 * cout)
    _check(y, "y", m * cin)
    _check(dy, "dy", m * cin)
    _check(dpk, "d_pointwise_kernel", cin * cout)
    ws, wsb = _ws(L.query("unet_pointwise_bwd_data_bnrelu_wgrad_workspace", m, cin, cout), da.device)
    _call("unet_pointwise_bwd_data_bnrelu_wgrad",
          (4.0 * m * cin * cout, 4.0 * (2 * m * cout + 2 * m * cin + 2 * cin * cout)),
          _ptr(da), _ptr(z), m, cin, cout, _ptr(pk), _ptr(scale), _ptr(shift), _ptr(coef), _ptr(y), _ptr(dy),
          _ptr(dpk), ws, wsb, _stream())


def image_block_bwd_wgrad(x: Tensor, n: int, h: int, w: int, wcin: int, cout: int, pk: Tensor, scale: Tensor,
                          shift: Tensor, coef: Tensor, da: Tensor, z: Tensor, y: Tensor, ddk: Tensor, dpk: Tensor):
    """Both weight gradients of the image block in one pass (unet_image_block_bwd_wgrad): x the
    (n, h, w, 4) zero-padded input, pk the padded (4, cout) kernel; ddk (3, 3, wcin, 1) and
    dpk (1, 1, wcin, cout) are written in the Keras shapes."""
    m = n * h * w
    _check(x, "x", m * 4)
    _check(da, "da", m * cout)
    _check(z, "z", m * cout)
    _check(y, "y", m * 4)
    _check(pk, "pointwise_kernel", 4 * cout)
    _check(coef, "coef", 3 * cout)
    _check(ddk, "d_depthwise_kernel", 9 * wcin)
    _check(dpk, "d_pointwise_kernel", wcin * cout)
    ws, wsb = _ws(L.query("unet_image_block_bwd_wgrad_workspace", n, h, w, cout), da.device)
    _call("unet_image_block_bwd_wgrad",
          (2.0 * m * 4 * cout + 2.0 * m * 4 * cout + 2.0 * m * 9 * 4,
           4.0 * (2 * m * cout + 2 * m * 4 + 4 * cout)),
          _ptr(x), n, h, w, wcin, cout, _ptr(pk), _ptr(scale), _ptr(shift), _ptr(coef), _ptr(da), _ptr(z), _ptr(y),
          _ptr(ddk), _ptr(dpk), ws, wsb, _stream())


# ------------------------------------------------------------ Conv2DTranspose ---
def conv_transpose2x2_fwd(x: View, n, h, w, cout, k: Tensor, b: Optional[Tensor], out: Tensor,
                          kx: Optional[Tensor] = None):
    """kx: k's split-precision planes in its own layout (split_x3(keep=True) of (4 cout, cin)): the
    bf16x6 GEMM (unet_conv_transpose2x2_fwd_x3) where cin % 32 == 0."""
    _check(k, "kernel", 4 * cout * x.c0)
    _check(out, "out", n * 4 * h * w * cout)
    vs = x.c_struct()
    m = n * h * w
    work = (8.0 * m * x.c0 * cout, 4.0 * (m * x.c0 + 4 * m * cout + 4 * x.c0 * cout))
    if _planes(kx, 4 * cout * x.c0, "conv_transpose2x2_fwd") is not None:
        _call("unet_conv_transpose2x2_fwd_x3", work, ctypes.byref(vs), n, h, w, cout, _ptr(k), _ptr(kx), _ptr(b),
              _ptr(out), _stream())
        return
    _call("unet_conv_transpose2x2_fwd", work, ctypes.byref(vs), n, h, w, cout, _ptr(k), _ptr(b), _ptr(out), _stream())


def conv_transpose2x2_bwd(x: View, n, h, w, cout, k: Tensor, dout: Tensor, dx: Optional[Tensor],
                          dk: Optional[Tensor], db: Optional[Tensor]):
    """Data gradient (dx) and/or weight + bias gradients (dk, db; both or neither)."""
    _check(dout, "dout", n * 4 * h * w * cout)
    if dk is not None:
        _check(dk, "dkernel", 4 * cout * x.c0)
        _check(db, "dbias", cout)
    if dx is not None:
        _check(dx, "dx", n * h * w * x.c0)
    ws, wsb = _ws(L.query("unet_conv_transpose2x2_bwd_workspace", n, h, w, x.c0, cout), dout.device)
    vs = x.c_struct()
    m = n * h * w
    fl = ((8.0 if dx is not None else 0.0) + (8.0 if dk is not None else 0.0)) * m * x.c0 * cout
    nb = ((16.0 * m * cout + 4.0 * m * x.c0 + 16.0 * x.c0 * cout if dx is not None else 0.0) +
          (x.src_bytes(n, h, w) + 16.0 * m * cout + 16.0 * x.c0 * cout if dk is not None else 0.0))
    _call("unet_conv_transpose2x2_bwd", (fl, nb), ctypes.byref(vs), n, h, w, cout, _ptr(k), _ptr(dout), _ptr(dx),
          _ptr(dk), _ptr(db), ws, wsb, _stream())


def conv_transpose2x2_bwd_data_bnstats_slabs(x: View, n, h, w, cout) -> int:
    """Slab count of conv_transpose2x2_bwd_data_bnstats's BN partials (0: no such path)."""
    vs = x.c_struct()
    return L.query("unet_conv_transpose2x2_bwd_data_bnstats_slabs", ctypes.byref(vs), n, h, w, cout)


def conv_transpose2x2_bwd_data_bnstats(x: View, n, h, w, cout, k: Tensor, dout: Tensor, dx: Tensor, mean, rstd,
                                       partials: Tensor, kxt: Optional[Tensor] = None):
    """Data gradient of conv_transpose2x2 (x: the BNRELU view of the block below, no dropout) that
    also emits that block's BN-backward partials (finish: bn_relu_bwd_stats_finish).  kxt: k's
    split-precision planes transposed (split_x3 of (4 cout, cin): [3][cin][4 cout]), the bf16x6 GEMM."""
    S = conv_transpose2x2_bwd_data_bnstats_slabs(x, n, h, w, cout)
    _check(dout, "dout", n * 4 * h * w * cout)
    _check(dx, "dx", n * h * w * x.c0)
    _check(partials, "bn_partials", bn_stats_partials_numel(S, x.c0))
    vs = x.c_struct()
    m = n * h * w
    nb = 16.0 * m * cout + 8.0 * m * x.c0 + 16.0 * x.c0 * cout + 8.0 * S * x.c0
    if _planes(kxt, 4 * cout * x.c0, "conv_transpose2x2_bwd_data_bnstats") is not None:
        _call("unet_conv_transpose2x2_bwd_data_bnstats_x3", (8.0 * m * x.c0 * cout, nb), ctypes.byref(vs), n, h, w,
              cout, _ptr(k), _ptr(kxt), _ptr(dout), _ptr(dx), _ptr(mean), _ptr(rstd), _ptr(partials), _stream())
        return
    _call("unet_conv_transpose2x2_bwd_data_bnstats", (8.0 * m * x.c0 * cout, nb), ctypes.byref(vs), n, h, w, cout,
          _ptr(k), _ptr(dout), _ptr(dx), _ptr(mean), _ptr(rstd), _ptr(partials), _stream())


# ---------------------------------------------------------------- head / loss ---
def head_fwd(x: View, n, h, w, ncls, k: Tensor, b: Optional[Tensor], prob: Tensor):
    _check(k, "kernel", x.c0 * ncls)
    _check(prob, "prob", n * h * w * ncls)
    vs = x.c_struct()
    _call("unet_head_fwd", (2.0 * n * h * w * x.c0 * ncls, x.src_bytes(n, h, w) + 4.0 * n * h * w * ncls),
          ctypes.byref(vs), n, h, w, ncls, _ptr(k), _ptr(b), _ptr(prob), _stream())


def dice_fwd(y_true: Tensor, y_pred: Tensor, n: int, hw: int, ncls: int, smooth: float, sums: Optional[Tensor],
             result: Tensor):
    _check(y_true, "y_true", n * hw * ncls)
    _check(y_pred, "y_pred", n * hw * ncls)
    _check(result, "result", 3)
    if sums is not None:
        _check(sums, "sums", n * ncls * 3)
    ws, wsb = _ws(L.query("unet_dice_workspace", n, hw, ncls), y_pred.device)
    _call("unet_dice_fwd", (4.0 * n * hw * ncls, 8.0 * n * hw * ncls), _ptr(y_true), _ptr(y_pred), n, hw, ncls, float(smooth), _ptr(sums), _ptr(result), ws,
           wsb, _stream())


def head_bwd(x: View, n, h, w, ncls, k: Tensor, prob: Tensor, y_true: Tensor, sums: Tensor, smooth: float,
             loss_kind: int, dx: Tensor, dk: Tensor, db: Tensor, loss_scale: float = 1.0):
    _check(prob, "prob", n * h * w * ncls)
    _check(y_true, "y_true", n * h * w * ncls)
    _check(dx, "dx", n * h * w * x.c0)
    ws, wsb = _ws(L.query("unet_head_bwd_workspace", n, h, w, x.c0, ncls), prob.device)
    vs = x.c_struct()
    m = n * h * w
    _call("unet_head_bwd", (4.0 * m * x.c0 * ncls, x.src_bytes(n, h, w) + 4.0 * m * (x.c0 + 2 * ncls)),
          ctypes.byref(vs), n, h, w, ncls, _ptr(k), _ptr(prob), _ptr(y_true), _ptr(sums),
          float(smooth), int(loss_kind), float(loss_scale), _ptr(dx), _ptr(dk), _ptr(db), ws, wsb, _stream())


def head_bwd_bnstats_slabs(x: View, n, h, w, ncls) -> int:
    vs = x.c_struct()
    return L.query("unet_head_bwd_bnstats_slabs", ctypes.byref(vs), n, h, w, ncls)


def head_bwd_bnstats(x: View, n, h, w, ncls, k: Tensor, prob: Tensor, y_true: Tensor, sums: Tensor, smooth: float,
                     loss_kind: int, dx: Optional[Tensor], dk: Tensor, db: Tensor, mean, rstd, partials: Tensor,
                     loss_scale: float = 1.0, dlogit: Optional[Tensor] = None):
    """head_bwd that also emits the BN-backward partials of the head input's block.  With dlogit
    (m,) instead of dx, only dL/dlogit per pixel is stored (dx = dlogit (x) kernel, rank one)."""
    S = head_bwd_bnstats_slabs(x, n, h, w, ncls)
    _check(prob, "prob", n * h * w * ncls)
    _check(y_true, "y_true", n * h * w * ncls)
    if (dx is None) == (dlogit is None):
        raise ValueError("head_bwd_bnstats: give dx or dlogit")
    if dx is not None:
        _check(dx, "dx", n * h * w * x.c0)
    else:
        _check(dlogit, "dlogit", n * h * w)
    _check(partials, "bn_partials", bn_stats_partials_numel(S, x.c0))
    ws, wsb = _ws(L.query("unet_head_bwd_workspace", n, h, w, x.c0, ncls), prob.device)
    vs = x.c_struct()
    m = n * h * w
    _call("unet_head_bwd_bnstats", (4.0 * m * x.c0 * ncls,
                                    x.src_bytes(n, h, w) + 4.0 * m * ((x.c0 if dx is not None else 1) + 2 * ncls)),
          ctypes.byref(vs), n, h, w, ncls, _ptr(k), _ptr(prob), _ptr(y_true), _ptr(sums), float(smooth),
          int(loss_kind), float(loss_scale), _ptr(dx), _ptr(dlogit), _ptr(dk), _ptr(db), _ptr(mean), _ptr(rstd),
          _ptr(partials), ws, wsb, _stream())


def meaniou_update(y_true: Tensor, y_pred: Tensor, num_classes: int, threshold: Optional[float],
                   confusion: Tensor):
    _check(y_true, "y_true")
    _check(y_pred, "y_pred", y_true.numel())
    if confusion.dtype != torch.int64 or confusion.numel() != num_classes * num_classes or not confusion.is_cuda:
        raise ValueError("confusion: expected an int64 device tensor of num_classes^2 counts")
    thr = -1.0 if threshold is None else float(threshold)
    if threshold is not None and threshold < 0:
        raise ValueError("threshold must be >= 0")
    _call("unet_meaniou_update", (0.0, 8.0 * y_true.numel()), _ptr(y_true), _ptr(y_pred), y_true.numel(), num_classes, thr, _ptr(confusion),
           _stream())


def adamw_step(param: Tensor, grad: Tensor, m: Tensor, v: Tensor, lr, wd, b1, b2, eps, alpha, grad_scale=1.0):
    n = param.numel()
    for t, nm in ((param, "param"), (grad, "grad"), (m, "m"), (v, "v")):
        _check(t, nm, n)
    _call("unet_adamw_step", (20.0 * n, 28.0 * n), _ptr(param), _ptr(grad), _ptr(m), _ptr(v), n, float(lr), float(wd), float(b1),
           float(b2), float(eps), float(alpha), float(grad_scale), _stream())
