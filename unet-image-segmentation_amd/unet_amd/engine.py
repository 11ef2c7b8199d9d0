"""The U-Net train / predict step on MI355X: a fixed schedule of libunet_hip.so kernels.

Replaces what Keras + TensorFlow do for the reference's hot path:
  forward   model/u_net.py:28-116 (U_NET), conv_block :5-26
  loss      utils/loss.py:9-48, utils/metrics.py:6-62
  backward  the GradientTape of `model.fit` (scripts/train.py:308)
  update    keras.optimizers.AdamW (scripts/train.py:226) -> optim.AdamW

Data layout in HBM (per GPU, batch N):
  * conv_block outputs are stored RAW (pre-BatchNorm z, NHWC); the BN affine + ReLU, the
    2x2 max-pool, the skip concat and dropout are applied by the consumer on load
    (activation views), so activations a = relu(bn(z)), pooled tensors and concat buffers
    are never materialised;
  * each block also keeps its depthwise output y (the pointwise weight gradient needs it);
  * trainable variables / gradients / Adam moments: one flat buffer each (params.py).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L
from . import ops
from .ops import View
from .params import FILTERS, VarSpec, check_input_size, count_params, flat_layout, init_weights, unet_variables

BN_EPS = 1e-3       # keras BatchNormalization default epsilon
BN_MOMENTUM = 0.99  # keras BatchNormalization default momentum
SMOOTH = 1e-7       # K.epsilon() (utils/metrics.py:4)
DROP_SITES = ("bneck_dropout", "dec4_dropout", "dec3_dropout", "dec2_dropout")


FUSE_MIN_PIXELS = 64 * 64  # fused conv forward from the 64 x 64 level up (tools/bench_sepconv.py sweeps)
# ... and on a smaller level once the batch gives it >= 128 pixel tiles: the 32 x 32 level from
# batch 16 (configs[1]; with the weight planes staged by LDS-DMA its bf16x6 launch 54.8 -> 47.3 us, and
# the step 10.44-10.47 -> 10.37-10.41 ms, profiles/r6h_fuse32_b16_ab.txt); at batch 8 (configs[4] per
# GPU) the split launches stay faster (6.05-6.07 vs 6.15-6.16 ms)
# (a fixed constant: every data-parallel rank takes the same route; an A/B sets the engine attributes
# fuse_min_pixels / fuse_min_total, bench.py --fuse-min-pixels / --fuse-min-total)
FUSE_MIN_TOTAL_PIXELS = 16 * 1024
# blocks whose weight gradients recompute y instead of the forward storing it: an output channel count
# (64: the fused block backward), or an (input, output) channel pair
RECOMPUTE_Y_COUTS = (64,)


def block_fwd_choice(view: View, n: int, h: int, w: int, cout: int, training: bool, fuse: str = "auto",
                     recompute_y: bool = True, recompute_couts=RECOMPUTE_Y_COUTS, min_total: int = FUSE_MIN_TOTAL_PIXELS,
                     min_pixels: int = FUSE_MIN_PIXELS):
    """The kernels a conv_block forward runs: (fused, keep_y).  fused: one unet_sepconv_fwd launch
    (else unet_dwconv3x3_fwd + unet_pointwise_fwd, which always store y); keep_y: the fused launch
    also stores the depthwise output y for the weight gradients (training blocks whose weight
    gradients do not recompute it).  Shared by the engine and bench.py's encoder table."""
    want = fuse == "always" or (fuse == "auto" and (h * w >= min_pixels or n * h * w >= min_total))
    if not (want and ops.sepconv_supported(view, n, h, w, cout)):
        return False, training
    y_recompute = training and recompute_y and (cout in recompute_couts or (view.channels, cout) in recompute_couts) and \
        ops.sepconv_bwd_filter_supported(view, n, h, w, cout)
    return True, training and not y_recompute


def _mix64(*vals: int) -> int:
    z = 0x243F6A8885A308D3
    for v in vals:
        z = (z ^ (int(v) & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF
        z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
    return z


@dataclass
class Block:
    """One conv_block (SeparableConv2D -> BatchNormalization -> ReLU)."""

    name: str
    cin: int    # channels the kernels see (the image block is padded to a multiple of 4)
    cout: int
    level: int  # spatial size = input / 2**level
    wcin: int = 0  # channels of the Keras weights when they differ from cin (padded block)


@dataclass
class BlockBufs:
    y: torch.Tensor
    z: torch.Tensor
    part: torch.Tensor
    mean: torch.Tensor
    rstd: torch.Tensor
    scale: torch.Tensor
    shift: torch.Tensor
    da: torch.Tensor  # gradient w.r.t. this block's output activation
    dz: Optional[torch.Tensor] = None  # backward-only, allocated on first backward
    dy: Optional[torch.Tensor] = None
    coef: Optional[torch.Tensor] = None  # BN-backward coefficients (mean, dbeta/M, rstd*dgamma/M)
    bnpart: Optional[torch.Tensor] = None  # BN-backward partial sums emitted by the producer of da
    bn_slabs: int = 0  # > 0: bnpart holds this many fresh slabs for the next backward of the block
    bn_masked: bool = False  # ... and they already carry the dropout mask between the block and its consumer
    bnpart_s: int = -1  # the slab count bnpart's counters were last laid out for
    y_recompute: bool = False  # last training forward kept no y: the weight grads recompute it
    zsel: Optional[torch.Tensor] = None  # encoder block2: the 2x2 max-pool selection of z (n, h/2, w/2, C)
    dlogit: Optional[torch.Tensor] = None  # last block, binary head: dL/dlogit per pixel (its da is rank one)
    dwpart: Optional[torch.Tensor] = None  # depthwise filter-gradient slabs of the fused data + filter pass
    da_rank1: bool = False  # this backward's da is dlogit (x) the head kernel, never materialised
    rec: Optional[torch.Tensor] = None  # SyncBN: this replica's (count, mean, M2) record, float64 1 + 2C
    recs: Optional[torch.Tensor] = None  # SyncBN: the gathered records [world][1 + 2C]
    bsums: Optional[torch.Tensor] = None  # SyncBN backward: [sum g | sum g*xhat] (2C), all-reduced


@dataclass
class Acts:
    n: int
    blocks: Dict[str, BlockBufs]
    up: Dict[str, torch.Tensor]
    dup: Dict[str, torch.Tensor]
    prob: torch.Tensor
    dz: torch.Tensor
    dy: torch.Tensor
    sums: torch.Tensor
    result: torch.Tensor
    xpad: Optional[torch.Tensor] = None  # channel-padded image (image block input)


class UNetEngine:
    """Device-resident U-Net with explicit forward / backward schedules."""

    def __init__(self, input_size: Sequence[int], num_classes: int = 1, dropout_rate: float = 0.2,
                 use_batch_norm: bool = True, filters: Sequence[int] = FILTERS, device=None, seed: int = 2301):
        self.h, self.w, self.c = check_input_size(input_size, len(filters))
        if num_classes < 1:
            raise ValueError("num_classes must be >= 1")
        if not 0.0 <= dropout_rate < 1.0:
            raise ValueError("dropout_rate must be in [0, 1)")
        if not torch.cuda.is_available():
            raise RuntimeError("UNetEngine needs a HIP device (MI355X); there is no CPU execution path")
        L.load()
        self.num_classes = int(num_classes)
        self.dropout_rate = float(dropout_rate)
        self.use_bn = bool(use_batch_norm)
        self.filters = tuple(int(f) for f in filters)
        self.device = torch.device(device if device is not None else "cuda")
        self.seed = int(seed)
        self.specs: List[VarSpec] = unet_variables(self.c, self.num_classes, self.use_bn, self.filters)
        self.spec_by_name = {s.name: s for s in self.specs}
        self.train_layout = flat_layout(self.specs, True)
        self.stat_layout = flat_layout(self.specs, False)
        self.params = torch.zeros(self.train_layout.total, dtype=torch.float32, device=self.device)
        self.grads = torch.zeros_like(self.params)
        self.stats = torch.zeros(self.stat_layout.total, dtype=torch.float32, device=self.device)
        self.vars: Dict[str, torch.Tensor] = {}
        self.gvars: Dict[str, torch.Tensor] = {}
        for s in self.specs:
            if s.trainable:
                o = self.train_layout.offsets[s.name]
                self.vars[s.name] = self.params[o:o + s.size].view(s.shape)
                self.gvars[s.name] = self.grads[o:o + s.size].view(s.shape)
            else:
                o = self.stat_layout.offsets[s.name]
                self.vars[s.name] = self.stats[o:o + s.size].view(s.shape)
        self.params_version = 0  # bumped whenever the trainable weights are replaced (set_weights / train_step)
        self.set_weights_dict(init_weights(self.specs, self.seed))
        self._build_plan()
        self._build_x3()
        self._acts: Dict[int, Acts] = {}
        self.step_count = 0
        self.rank_salt = 0  # data-parallel rank (dropout streams); set by model.enable_data_parallel
        self.grad_hook: Optional[Callable[[int], None]] = None  # called with a flat-offset low-water mark
        # Off-critical-path backward work (weight gradients of the pointwise, depthwise and
        # transposed convolutions) runs on a second HIP stream, overlapping the data-gradient
        # chain on the main stream.
        lo_prio, hi_prio = torch.cuda.Stream.priority_range()
        self.main = torch.cuda.Stream(device=self.device, priority=hi_prio)
        self.side = torch.cuda.Stream(device=self.device, priority=lo_prio)
        self.overlap = os.environ.get("UNET_OVERLAP", "1") != "0"  # 0: single stream (clean profiles)
        # Fused depthwise+pointwise forward (unet_sepconv_fwd) vs the two launches: "auto" uses it
        # where it measured faster (levels of >= 64x64 pixels, tools/bench_sepconv.py and
        # profiles/r1i_sepconv_bn_sweep.log); "always" / "never" force the choice (tests).
        self.fuse_sepconv = "auto"
        self.fuse_min_pixels = FUSE_MIN_PIXELS  # levels of at least this many pixels per image ...
        self.fuse_min_total = FUSE_MIN_TOTAL_PIXELS  # ... and below that from this many pixels per launch
        # BN + ReLU backward folded into the pointwise data-gradient GEMM (no separate dz pass)
        self.fuse_bn_bwd = True
        # BN-backward statistics of a block emitted by the launch that completes its da (the next
        # block's depthwise data gradient through BN+ReLU or the max-pool, the Conv2DTranspose data
        # gradient, the head), not by a separate pass over (da, z)
        self.fuse_bn_stats = True
        # image block (4 padded channels): data and pointwise weight gradient in one streaming pass over
        # (da, z, y) that forms dz on the fly, so dz (M x 64) is neither stored nor re-read
        self.img_fused_wgrad = True
        # ... and, with no data gradient to produce (the network's input), its depthwise kernel
        # gradient in the same pass: dy is contracted with x's 3x3 neighbourhood as it is formed,
        # never stored (unet_image_block_bwd_wgrad; one launch + reductions instead of four)
        self.img_fused_dwf = os.environ.get("UNET_IMG_DWF", "1") != "0"
        # weight gradients of the HBM-bound 64 -> 64 blocks in one pass that recomputes the
        # depthwise output y from the block's input view (unet_sepconv_bwd_filter), so their
        # forward never stores y
        self.recompute_y = os.environ.get("UNET_RECOMPUTE_Y", "1") != "0"
        self.recompute_y_couts = RECOMPUTE_Y_COUTS
        # issue a y-recomputing block's fused weight gradient (one 111 KB-LDS block per CU for the
        # launch's whole length) only after the main stream has issued the NEXT block's statistics
        # finish, instead of beside its own depthwise data gradient (under data parallelism the
        # all-reduce low-water report waits for the deferred launch, see _grads_ready)
        self.defer_sw = os.environ.get("UNET_SW_DEFER", "1") != "0"
        # the y-recomputing 64-output blocks run their whole backward but the depthwise data
        # gradient as ONE main-stream pass (unet_sepconv_bwd_fused: dz formed per tile, dy and both
        # weight gradients from it; dz never stored) instead of the data-gradient GEMM + the
        # side-stream weight-gradient pass
        self.fuse_block_bwd = True
        # a BN+ReLU-view block's depthwise FILTER gradient accumulated by its depthwise data-gradient pass
        # (the same dy window, x from the z the BN statistics read): no second pass over dy and the view
        # on the side stream; the per-tile slabs are summed there instead (round 6)
        self.dw_fused_filter = True
        # SyncBN (SURVEY 8(e) option, off by default like tf.distribute / Keras synchronized=False):
        # under data parallelism every BatchNorm uses the global batch's statistics -- the forward
        # gathers each replica's (count, mean, M2) and combines them in rank order, the backward
        # all-reduces (sum g, sum g*xhat) before dz is formed.  Set by model.enable_data_parallel.
        self.sync_bn = False
        self.sync_group = None
        self.sync_world = 1
        self.sync_global_n = 0  # images in the global batch of the current step (model.train_step)
        # inference forward captured as a HIP graph per input shape (hipGraph through torch.cuda.CUDAGraph):
        # one graph launch replays the forward's ~60 kernel launches, so small-batch inference is not
        # bound by the host's per-launch cost.  Opt-in (UNET_GRAPH_PREDICT=1 or this attribute).
        self.graph_predict = os.environ.get("UNET_GRAPH_PREDICT", "0") == "1"
        self._pgraphs: Dict[tuple, tuple] = {}
        self._pending_side = None
        self._pending_ready: Optional[str] = None
        self._ev = None  # created on first use (on the device)

    # ------------------------------------------------------------------ weights ------
    def set_weights_dict(self, weights: Dict[str, np.ndarray]) -> None:
        for name, arr in weights.items():
            if name not in self.vars:
                raise KeyError(f"unknown variable {name}")
            t = self.vars[name]
            a = np.asarray(arr, dtype=np.float32)
            if tuple(a.shape) != tuple(t.shape):
                raise ValueError(f"{name}: shape {a.shape} != {tuple(t.shape)}")
            t.copy_(torch.from_numpy(np.ascontiguousarray(a)).to(self.device))

        self.params_version += 1

    def _build_x3(self):
        """Split-precision planes (ops.split_x3) of the pointwise kernels of the blocks whose fused
        forward can run the bf16x6 register-A kernel (channels % 16 == 0, >= 64): one launch per
        weight update refreshes the ones the forward's batch fuses (_refresh_x3)."""
        self.use_x3 = True
        self.x3_off: Dict[str, int] = {}
        self.x3_cand = []  # (block, segment) in block order
        off = 0
        for b in self.blocks:
            if b.cin % 16 == 0 and b.cin >= 64 and not b.wcin:
                src = self.train_layout.offsets[f"{b.name}_sepconv/pointwise_kernel"]
                self.x3_cand.append((b, (src, b.cin, b.cout, off)))
                self.x3_off[b.name] = off
                off += (3 * b.cin * b.cout + 7) // 8 * 8
        self.x3_live: set = set()
        self._x3_plans: Dict[int, tuple] = {}
        # ... and the same kernels' planes in their own layout ([3][Cin][Cout], k = Cout contiguous)
        # for the split-precision BatchNorm-backward data gradient (unet_pointwise_bwd_data_bnrelu_x3),
        # refreshed by one launch per training forward: every block but the padded image block (the
        # 64-output blocks that take the fused block backward do not read theirs)
        self.x6_gemm = True
        self.x3d_off: Dict[str, int] = {}
        self.x3d_segs = []
        offd = 0
        for b in self.blocks:
            if b.cout % 32 == 0 and b.cin % 4 == 0 and not b.wcin:
                src = self.train_layout.offsets[f"{b.name}_sepconv/pointwise_kernel"]
                self.x3d_segs.append((src, b.cin, b.cout, offd))
                self.x3d_off[b.name] = offd
                offd += (3 * b.cin * b.cout + 7) // 8 * 8
        # the Conv2DTranspose kernels (2, 2, f, cin) seen as (4 f, cin): planes in their own layout for
        # the forward (k = cin contiguous) and transposed ([3][cin][4 f]) for the data gradient
        self.x3u_off: Dict[str, tuple] = {}
        self.x3t_segs = []
        offt = 0
        for stage, fi, cin, _b1, _b2 in self.dec:
            src = self.train_layout.offsets[f"{stage}_upsample/kernel"]
            self.x3d_segs.append((src, 4 * fi, cin, offd))
            self.x3t_segs.append((src, 4 * fi, cin, offt))
            self.x3u_off[stage] = (offd, offt, 12 * fi * cin)
            offd += (12 * fi * cin + 7) // 8 * 8
            offt += (12 * fi * cin + 7) // 8 * 8
        # one arena, so a training forward refreshes all three plane sets in ONE unet_split_x3_mixed launch
        off, offd, offt = (max(v, 8) for v in (off, offd, offt))
        self.x3buf = torch.empty(off + offd + offt, dtype=torch.int16, device=self.device)
        self.pkx = self.x3buf[:off]
        self.pkd = self.x3buf[off:off + offd]
        self.pkt = self.x3buf[off + offd:]
        self.x3_mixed = [(so, r, c, do + off, 1) for so, r, c, do in self.x3d_segs] + \
                        [(so, r, c, do + off + offd, 0) for so, r, c, do in self.x3t_segs]

    def _refresh_x3(self, n: int, training: bool = False):
        """Re-split on EVERY forward (one small launch): the planes then always match the fp32
        weights the backward reads, whatever wrote engine.params in between (AdamW, a custom
        optimizer loop, an in-place edit of engine.vars, a data-parallel broadcast).  Only the
        blocks whose level the batch of n images fuses (block_fwd_choice's pixel rule)."""
        # (a training step with the split-precision GEMMs also refreshes the blocks whose forward is the
        # depthwise launch + the pointwise GEMM -- unet_pointwise_fwd_x3 reads the same planes -- and the
        # rows GEMMs' own planes, pkd / pkt: one mixed-layout launch for all of them)
        six = training and self.x6_gemm
        key = (n, self.fuse_min_pixels, self.fuse_min_total, six, self.use_x3)
        plan = self._x3_plans.get(key)
        if plan is None:  # (cached per batch size: the host loop is on the critical path of small steps)
            segs, live = [], set()
            if self.use_x3:
                for b, seg in self.x3_cand:
                    h, w = self._dims(b.level)
                    if six or h * w >= self.fuse_min_pixels or n * h * w >= self.fuse_min_total:
                        segs.append(seg + (0,))
                        live.add(b.name)
            if six:
                segs += self.x3_mixed
            plan = self._x3_plans[key] = (segs, live)
        segs, self.x3_live = plan
        if segs:
            ops.split_x3(self.params, segs, self.x3buf)

    def _ukx(self, stage: str, training: bool):
        """The training forward's split-precision planes of an upsample kernel (None: fp32 route)."""
        if not (self.x6_gemm and training):
            return None
        o, _, nel = self.x3u_off[stage]
        return self.pkd[o:o + nel]

    def _ukt(self, stage: str):
        if not self.x6_gemm:
            return None
        _, o, nel = self.x3u_off[stage]
        return self.pkt[o:o + nel]

    def _pkd(self, b: "Block"):
        o = self.x3d_off.get(b.name) if self.x6_gemm else None
        return None if o is None else self.pkd[o:o + 3 * b.cin * b.cout]

    def _pkx(self, b: "Block"):
        o = self.x3_off.get(b.name) if self.use_x3 and b.name in self.x3_live else None
        return None if o is None else self.pkx[o:o + 3 * b.cin * b.cout]

    def get_weights_dict(self) -> Dict[str, np.ndarray]:
        return {s.name: self.vars[s.name].detach().cpu().numpy().copy() for s in self.specs}

    def count_params(self):
        return count_params(self.specs)

    # --------------------------------------------------------------------- plan ------
    def _build_plan(self):
        f = self.filters
        self.enc: List[tuple] = []
        c = self.c
        # The image block runs on a channel-padded copy of the input (3 -> 4 channels, zero
        # padding), so every kernel takes its vectorised / fused path; its Keras-shaped weights
        # are mirrored into padded buffers each forward and the gradients copied back.
        self.cpad = c if c % 4 == 0 else (c + 3) // 4 * 4
        for i, fi in enumerate(f):
            b1 = Block(f"enc{i + 1}_block1", c, fi, i) if i > 0 or self.cpad == c else \
                Block(f"enc{i + 1}_block1", self.cpad, fi, i, wcin=c)
            b2 = Block(f"enc{i + 1}_block2", fi, fi, i)
            self.enc.append((f"enc{i + 1}", b1, b2))
            c = fi
        d = len(f)
        bn = 2 * f[-1]
        self.bneck = (Block("bneck_block1", c, bn, d), Block("bneck_block2", bn, bn, d))
        self.dec: List[tuple] = []
        c = bn
        for i, fi in enumerate(reversed(f)):
            stage = len(f) - i
            lvl = stage - 1
            self.dec.append((f"dec{stage}", fi, c, Block(f"dec{stage}_block1", 2 * fi, fi, lvl),
                             Block(f"dec{stage}_block2", fi, fi, lvl)))
            c = fi
        self.blocks: List[Block] = [b for _, b1, b2 in self.enc for b in (b1, b2)] + list(self.bneck) + \
                                   [b for *_, b1, b2 in self.dec for b in (b1, b2)]

    def _dims(self, level: int):
        return self.h >> level, self.w >> level

    def acts(self, n: int) -> Acts:
        a = self._acts.get(n)
        if a is not None:
            return a
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        blocks = {}
        max_in = max_out = 0
        for b in self.blocks:
            h, w = self._dims(b.level)
            m = n * h * w
            max_in = max(max_in, m * b.cin)
            max_out = max(max_out, m * b.cout)
            blocks[b.name] = BlockBufs(
                y=torch.empty((n, h, w, b.cin), **f32), z=torch.empty((n, h, w, b.cout), **f32),
                part=torch.zeros(ops.bn_partials_numel(m, b.cout), **f32),
                mean=torch.zeros(b.cout, **f32), rstd=torch.zeros(b.cout, **f32),
                scale=torch.zeros(b.cout, **f32), shift=torch.zeros(b.cout, **f32),
                da=torch.empty((n, h, w, b.cout), **f32))
        for _, _, b2 in self.enc:  # the pooled stage outputs: their consumers read one value per window
            h, w = self._dims(b2.level)
            blocks[b2.name].zsel = torch.empty((n, h // 2, w // 2, b2.cout), **f32)
        up, dup = {}, {}
        for stage, fi, cin, b1, b2 in self.dec:
            h, w = self._dims(b1.level)
            up[stage] = torch.empty((n, h, w, fi), **f32)
            dup[stage] = torch.empty((n, h, w, fi), **f32)
        a = Acts(n=n, blocks=blocks, up=up, dup=dup,
                 prob=torch.empty((n, self.h, self.w, self.num_classes), **f32),
                 dz=torch.empty(max_out, **f32), dy=torch.empty(max_in, **f32),
                 sums=torch.zeros(n * self.num_classes * 3, **f32), result=torch.zeros(3, **f32))
        self._acts[n] = a
        return a

    def release_buffers(self):
        self._pgraphs.clear()  # (the captured inference graphs read these buffers)
        self._acts.clear()

    # ------------------------------------------------------------------ forward ------
    def _bn(self, name):
        if self.use_bn:
            return (self.vars[f"{name}_bn/gamma"], self.vars[f"{name}_bn/beta"], self.vars[f"{name}_bn/moving_mean"],
                    self.vars[f"{name}_bn/moving_variance"])
        return None, self.vars[f"{name}_sepconv/bias"], None, None

    def _block_fwd(self, A: Acts, b: Block, view: View, training: bool) -> View:
        n = A.n
        h, w = self._dims(b.level)
        m = n * h * w
        bb = A.blocks[b.name]
        gamma, beta, mm, mv = self._bn(b.name)
        dk, pk = self._wts(b)
        fused, keep_y = block_fwd_choice(view, n, h, w, b.cout, training, self.fuse_sepconv, self.recompute_y,
                                         self.recompute_y_couts, self.fuse_min_total, self.fuse_min_pixels)
        if fused:
            # one kernel: depthwise taps computed into the GEMM's A tile; y kept for the weight
            # grads unless they recompute it from the view
            stats = training and self.use_bn
            bb.y_recompute = training and not keep_y
            ops.sepconv_fwd(view, n, h, w, dk, b.cout, pk, bb.y if keep_y else None, bb.z,
                            bb.part if stats else None, bb.zsel, gamma, self._pkx(b))
            if stats:
                self._bn_finalize(bb, m, b.cout, gamma, beta, mm, mv)
            else:
                ops.bn_infer_params(gamma, beta, mm, mv, b.cout, BN_EPS, bb.scale, bb.shift)
            return View.bnrelu(bb.z, bb.scale, bb.shift)
        bb.y_recompute = False
        ops.dwconv3x3_fwd(view, n, h, w, dk, bb.y)
        if training and self.use_bn:
            ops.pointwise_fwd(bb.y, m, b.cin, b.cout, pk, bb.z, bb.part, pkx=self._pkx(b))
        else:
            ops.pointwise_fwd(bb.y, m, b.cin, b.cout, pk, bb.z, None, pkx=self._pkx(b))
        if bb.zsel is not None:
            ops.pool_select(bb.z, n, h, w, b.cout, gamma, bb.zsel)
        if training and self.use_bn:
            self._bn_finalize(bb, m, b.cout, gamma, beta, mm, mv)
        else:
            ops.bn_infer_params(gamma, beta, mm, mv, b.cout, BN_EPS, bb.scale, bb.shift)
        return View.bnrelu(bb.z, bb.scale, bb.shift)

    def _sync_bn_on(self) -> bool:
        return self.sync_bn and self.sync_world > 1 and self.use_bn

    def _bn_finalize(self, bb: BlockBufs, m: int, c: int, gamma, beta, mm, mv):
        """The training BatchNorm statistics of a block from its producer's partials: this replica's
        batch (unet_bn_finalize), or with SyncBN the global batch (records gathered over the group
        and combined in rank order on every replica: unet_bn_moments / unet_bn_finalize_moments)."""
        if not self._sync_bn_on():
            ops.bn_finalize(bb.part, m, c, gamma, beta, BN_EPS, BN_MOMENTUM, mm, mv, True, bb.mean, bb.rstd,
                            bb.scale, bb.shift)
            return
        import torch.distributed as dist
        if bb.rec is None or bb.rec.numel() != 1 + 2 * c:
            bb.rec = torch.empty(1 + 2 * c, dtype=torch.float64, device=self.device)
            bb.recs = torch.empty(self.sync_world * (1 + 2 * c), dtype=torch.float64, device=self.device)
        ops.bn_moments(bb.part, m, c, bb.rec)
        dist.all_gather_into_tensor(bb.recs, bb.rec, group=self.sync_group)
        ops.bn_finalize_moments(bb.recs, self.sync_world, c, gamma, beta, BN_EPS, BN_MOMENTUM, mm, mv, True,
                                bb.mean, bb.rstd, bb.scale, bb.shift)

    def _sync_bn_coef(self, bb: BlockBufs, b: Block, h: int, w: int, dgamma, dbeta):
        """SyncBN backward: coef from the group's (sum g, sum g*xhat) over the global batch; the
        replica's own dgamma / dbeta (its local sums) are left for the gradient all-reduce."""
        import torch.distributed as dist
        c = b.cout
        if bb.bsums is None:
            bb.bsums = torch.empty(2 * c, dtype=torch.float32, device=self.device)
        ops.copy_strided(dbeta, 1, c, c, bb.bsums, c)
        ops.copy_strided(dgamma, 1, c, c, bb.bsums[c:], c)
        dist.all_reduce(bb.bsums, group=self.sync_group)
        ops.bn_bwd_coef(bb.bsums, self.sync_global_n * h * w, c, True, bb.mean, bb.rstd, bb.coef)

    def _wts(self, b: Block, refresh: bool = True):
        """(depthwise, pointwise) kernels of a block as the kernels see them.  refresh=False (the
        backward of the forward that filled them) skips re-mirroring the padded image-block copy."""
        dk = self.vars[f"{b.name}_sepconv/depthwise_kernel"]
        pk = self.vars[f"{b.name}_sepconv/pointwise_kernel"]
        if not b.wcin:
            return dk, pk
        pad = self._pad_w
        if refresh:  # (3, 3, wcin, 1) -> (3, 3, cin, 1); (1, 1, wcin, cout) -> the first wcin rows
            ops.copy_strided(dk, 9, b.wcin, b.wcin, pad["dk"], b.cin)
            ops.copy_strided(pk, 1, b.wcin * b.cout, b.wcin * b.cout, pad["pk"], b.cin * b.cout)
        return pad["dk"], pad["pk"]

    def _gwts(self, b: Block):
        """(depthwise, pointwise) gradient buffers the kernels write for a block."""
        if not b.wcin:
            return self.gvars[f"{b.name}_sepconv/depthwise_kernel"], self.gvars[f"{b.name}_sepconv/pointwise_kernel"]
        return self._pad_w["gdk"], self._pad_w["gpk"]

    @property
    def _pad_w(self):
        p = getattr(self, "_pad_w_bufs", None)
        if p is None:
            b = self.blocks[0]
            z = dict(dtype=torch.float32, device=self.device)
            p = {"dk": torch.zeros((3, 3, b.cin, 1), **z), "pk": torch.zeros((1, 1, b.cin, b.cout), **z),
                 "gdk": torch.zeros((3, 3, b.cin, 1), **z), "gpk": torch.zeros((1, 1, b.cin, b.cout), **z)}
            self._pad_w_bufs = p
        return p

    def _padded_input(self, A: Acts, x: torch.Tensor) -> torch.Tensor:
        """The image with its channels zero-padded to self.cpad (a persistent buffer per batch)."""
        if self.cpad == self.c:
            return x
        xp = getattr(A, "xpad", None)
        if xp is None or xp.shape[0] != x.shape[0]:
            xp = torch.zeros((x.shape[0], self.h, self.w, self.cpad), dtype=torch.float32, device=self.device)
            A.xpad = xp
        ops.copy_strided(x, x.shape[0] * self.h * self.w, self.c, self.c, xp, self.cpad)
        return xp

    def drop_seeds(self, step: int) -> Dict[str, int]:
        """Dropout seeds of a step, per site; data-parallel ranks salt them with their rank so the
        replicas draw independent masks (rank_salt 0 = the single-process stream)."""
        if self.rank_salt:
            return {s: _mix64(self.seed, step, i + 1, self.rank_salt) for i, s in enumerate(DROP_SITES)}
        return {s: _mix64(self.seed, step, i + 1) for i, s in enumerate(DROP_SITES)}

    def forward(self, x: torch.Tensor, training: bool = False, seeds: Optional[Dict[str, int]] = None) -> torch.Tensor:
        """Forward pass (model/u_net.py:55-112).  x: (N, H, W, C) float32 NHWC on the device.
        training=True uses batch statistics (and updates the moving ones) and dropout."""
        if x.dim() != 4 or tuple(x.shape[1:]) != (self.h, self.w, self.c):
            raise ValueError(f"expected input (N, {self.h}, {self.w}, {self.c}), got {tuple(x.shape)}")
        x = x.contiguous()
        n = x.shape[0]
        A = self.acts(n)
        drop = training and self.dropout_rate > 0.0
        if drop and seeds is None:
            seeds = self.drop_seeds(self.step_count + 1)
        x = self._padded_input(A, x)
        self._refresh_x3(n, training)
        self._x_fwd = x
        v = View.plain(x)
        for stage, b1, b2 in self.enc:
            v = self._block_fwd(A, b1, v, training)
            self._block_fwd(A, b2, v, training)
            bb = A.blocks[b2.name]
            # MaxPooling2D (model/u_net.py:69) read as a BN+ReLU view of the window selections
            v = View.bnrelu(bb.zsel, bb.scale, bb.shift)
        v = self._block_fwd(A, self.bneck[0], v, training)
        v = self._block_fwd(A, self.bneck[1], v, training)
        if drop:
            v = v.dropout(self.dropout_rate, seeds["bneck_dropout"])
        for i, (stage, fi, cin, b1, b2) in enumerate(self.dec):
            h, w = self._dims(b1.level + 1)
            ops.conv_transpose2x2_fwd(v, n, h, w, fi, self.vars[f"{stage}_upsample/kernel"],
                                      self.vars[f"{stage}_upsample/bias"], A.up[stage], kx=self._ukx(stage, training))
            skip = A.blocks[self.enc[len(self.enc) - 1 - i][2].name]
            v = View.concat(A.up[stage], skip.z, skip.scale, skip.shift)
            if drop and i < len(self.dec) - 1:
                v = v.dropout(self.dropout_rate, seeds[f"{stage}_dropout"])
            v = self._block_fwd(A, b1, v, training)
            v = self._block_fwd(A, b2, v, training)
        ops.head_fwd(v, n, self.h, self.w, self.num_classes, self.vars["output_mask/kernel"],
                     self.vars["output_mask/bias"], A.prob)
        self._last_seeds = seeds
        return A.prob

    def loss(self, y_true: torch.Tensor, n: int) -> torch.Tensor:
        """dice_loss / dice_coef / iou_coef of the last forward -> result[0:3] (device)."""
        A = self.acts(n)
        ops.dice_fwd(y_true, A.prob, n, self.h * self.w, self.num_classes, SMOOTH, A.sums, A.result)
        return A.result

    # ----------------------------------------------------------------- backward ------
    def _event(self):
        if self._ev is None:
            self._ev = ops.DeviceEvent()
        return self._ev

    def _side_wait_main(self):
        main = torch.cuda.current_stream(self.device)
        if self._event() is None:
            self.side.wait_stream(main)
        else:
            self._ev.wait(self.side, main)

    def _main_wait_side(self):
        main = torch.cuda.current_stream(self.device)
        if self._event() is None:
            main.wait_stream(self.side)
        else:
            self._ev.wait(main, self.side)

    def run_beside(self, fn):
        """Run fn's launches on the side stream after the main stream's work so far (inline when
        single-stream).  The backward ends with the main stream waiting for the side stream, so
        the step's result includes them."""
        if not self.overlap:
            fn()
            return
        self._side_wait_main()
        with torch.cuda.stream(self.side):
            fn()

    def _flush_side(self):
        """Issue the deferred side-stream weight gradients (UNET_SW_DEFER), if any, then report
        the gradient low-water mark that waited for them."""
        if self._pending_side is not None:
            fn, self._pending_side = self._pending_side, None
            self._side_wait_main()
            with torch.cuda.stream(self.side):
                fn()
            name, self._pending_ready = self._pending_ready, None
            if name is not None:
                self._grads_ready(name)

    def _grads_ready(self, name: str):
        """Gradients at flat offsets >= offset(name) are final once both streams get here:
        the hook (bucketed all-reduce) is issued from the side stream after it has caught up
        with the main stream.  While a block's weight gradients are deferred the report waits
        for them (_flush_side), so no bucket is reduced before its last writer is issued."""
        if self.grad_hook is not None:
            if self._pending_side is not None:
                # keep the LOWEST flat offset reported while the deferral is pending (reports
                # arrive in descending-offset order today, but the hook must not depend on it)
                off = self.train_layout.offsets
                if self._pending_ready is None or off[name] < off[self._pending_ready]:
                    self._pending_ready = name
                return
            if self.overlap:
                self._side_wait_main()
                with torch.cuda.stream(self.side):
                    self.grad_hook(self.train_layout.offsets[name])
            else:
                self.grad_hook(self.train_layout.offsets[name])

    def _bnpart(self, tb: BlockBufs, S: int, c: int) -> torch.Tensor:
        """tb's producer-side BN-backward partials buffer sized for S slabs.  Its arrival counters
        sit at an S-dependent offset (lastblock.h), so a buffer last used with another S is
        re-zeroed, not just reused."""
        need = ops.bn_stats_partials_numel(S, c)
        if tb.bnpart is None or tb.bnpart.numel() < need:
            tb.bnpart = torch.zeros(need, dtype=torch.float32, device=self.device)
        elif tb.bnpart_s != S:
            tb.bnpart.zero_()
        tb.bnpart_s = S
        return tb.bnpart[:need]

    def _block_bwd(self, A: Acts, b: Block, view_in: View, dx0, dx1=None, drop_rate=0.0, drop_seed=0,
                   stats_target: Optional[BlockBufs] = None, view_f: Optional[View] = None):
        """Backward of one conv_block.  stats_target: the block whose output view_in reads (through
        BN+ReLU or the max-pool) when this launch completes its da (dx0); the depthwise data
        gradient then also emits that block's BN-backward partials.  view_f: the same input as
        view_in for the weight gradients when it reads cheaper (a max-pool input as the BN+ReLU
        view of its window selections; the data gradient routes through the POOL view of z)."""
        view_f = view_in if view_f is None else view_f
        n = A.n
        h, w = self._dims(b.level)
        m = n * h * w
        bb = A.blocks[b.name]
        if bb.dz is None:
            bb.dz = torch.empty(m * b.cout, dtype=torch.float32, device=self.device)
            bb.dy = torch.empty(m * b.cin, dtype=torch.float32, device=self.device)
            bb.coef = torch.empty(3 * b.cout, dtype=torch.float32, device=self.device)
        dz, dy = bb.dz, bb.dy
        if self.use_bn:
            dgamma, dbeta = self.gvars[f"{b.name}_bn/gamma"], self.gvars[f"{b.name}_bn/beta"]
        else:
            dgamma, dbeta = None, self.gvars[f"{b.name}_sepconv/bias"]
        dk, pk = self._wts(b, refresh=False)
        img_wg = img_all = False
        fused_bwd = self._fused_bwd(b, bb, drop_rate)
        if bb.da_rank1 and not fused_bwd:
            raise RuntimeError(f"{b.name}: rank-one da without the fused block backward")
        if self.fuse_bn_bwd and b.cin % 4 == 0 and b.cout % 4 == 0:
            # BN + ReLU backward statistics, then dz formed inside the data-gradient GEMM's loads
            if bb.bn_slabs and (drop_rate == 0.0 or bb.bn_masked):  # partials emitted by the producer of da
                ops.bn_relu_bwd_stats_finish(bb.bnpart[:ops.bn_stats_partials_numel(bb.bn_slabs, b.cout)],
                                             bb.bn_slabs, m, b.cout, bb.mean, bb.rstd, self.use_bn, dgamma, dbeta,
                                             bb.coef)
            else:
                ops.bn_relu_bwd_stats(bb.da, bb.z, m, b.cout, bb.mean, bb.rstd, bb.scale, bb.shift, self.use_bn,
                                      drop_rate, drop_seed, dgamma, dbeta, bb.coef)
            bb.bn_slabs = 0
            bb.bn_masked = False
            if self._sync_bn_on():
                self._sync_bn_coef(bb, b, h, w, dgamma, dbeta)
            self._flush_side()
            img_wg = self.img_fused_wgrad and drop_rate == 0.0 and b.cin == 4 and b.cout in (32, 64)
            img_all = (img_wg and self.img_fused_dwf and dx0 is None and view_f.mode == L.VIEW_PLAIN
                       and view_f.c0 == 4)
            if img_all:  # image block: both weight gradients in one pass, neither dz nor dy stored
                ops.image_block_bwd_wgrad(view_f.src0, n, h, w, b.wcin or b.cin, b.cout, pk, bb.scale, bb.shift,
                                          bb.coef, bb.da, bb.z, bb.y,
                                          self.gvars[f"{b.name}_sepconv/depthwise_kernel"],
                                          self.gvars[f"{b.name}_sepconv/pointwise_kernel"])
            elif img_wg:  # 4-channel image block: data + weight gradient in one pass, dz never stored
                ops.pointwise_bwd_data_bnrelu_wgrad(bb.da, bb.z, m, b.cin, b.cout, pk, bb.scale, bb.shift, bb.coef,
                                                    bb.y, dy, self._gwts(b)[1])
            elif fused_bwd:  # dy and both weight gradients in one pass over (da, z, the input view)
                gdk_f, gpk_f = self._gwts(b)
                if bb.da_rank1:  # the binary head's da = dlogit (x) kernel, formed on load
                    ops.sepconv_bwd_fused(view_f, n, h, w, dk, pk, None, bb.z, bb.scale, bb.shift, bb.coef, b.cout,
                                          dy, gdk_f, gpk_f, da_rank1=(bb.dlogit, self.vars["output_mask/kernel"]))
                    bb.da_rank1 = False
                else:
                    ops.sepconv_bwd_fused(view_f, n, h, w, dk, pk, bb.da, bb.z, bb.scale, bb.shift, bb.coef, b.cout,
                                          dy, gdk_f, gpk_f)
            else:
                ops.pointwise_bwd_data_bnrelu(bb.da, bb.z, m, b.cin, b.cout, pk, bb.scale, bb.shift, bb.coef,
                                              drop_rate, drop_seed, dy, dz, pkd=self._pkd(b))
        else:
            if self._sync_bn_on():
                raise RuntimeError("SyncBN needs the fused BN-backward route (fuse_bn_bwd, channels % 4 == 0)")
            ops.bn_relu_bwd(bb.da, bb.z, m, b.cout, bb.mean, bb.rstd, bb.scale, bb.shift, self.use_bn, drop_rate,
                            drop_seed, dgamma, dbeta, dz)
            ops.pointwise_bwd_data(dz, m, b.cin, b.cout, pk, dy)
        gdk, gpk = self._gwts(b)
        # the depthwise filter gradient from the data-gradient pass (unet_dwconv3x3_bwd_data_bnstats_dwf)
        dwf = (self.dw_fused_filter and dx0 is not None and stats_target is not None and self.fuse_bn_stats
               and self.fuse_bn_bwd and view_in.mode == L.VIEW_BNRELU and view_in.drop_rate == 0.0
               and view_f is view_in and not fused_bwd and not img_all and not bb.y_recompute and not b.wcin
               and ops.dwconv3x3_bwd_data_bnstats_slabs(view_in, n, h, w) > 0)

        def weight_grads():
            if fused_bwd or img_all:  # (done by the fused pass)
                return
            if bb.y_recompute:  # both kernels' gradients in one pass, y recomputed from view_in
                ops.sepconv_bwd_filter(view_f, n, h, w, dk, dy, dz, b.cout, gdk, gpk)
                return
            if not img_wg:  # (the image block's was accumulated by its data-gradient pass)
                ops.pointwise_bwd_filter(bb.y, dz, m, b.cin, b.cout, gpk)
            if not dwf:
                ops.dwconv3x3_bwd_filter(view_f, n, h, w, dy, gdk)
            if b.wcin:  # padded image block: keep the Keras-shaped slices
                ops.copy_strided(gpk, 1, b.wcin * b.cout, b.cin * b.cout,
                                 self.gvars[f"{b.name}_sepconv/pointwise_kernel"], b.wcin * b.cout)
                ops.copy_strided(gdk, 9, b.wcin, b.cin, self.gvars[f"{b.name}_sepconv/depthwise_kernel"], b.wcin)

        # the image block (dx0 None) has no data gradient after this: its weight gradients run
        # on the otherwise idle main stream, beside the side stream's enc1_block2 tail
        if fused_bwd:
            pass
        elif self.overlap and dx0 is not None:
            self._flush_side()
            if self.defer_sw and bb.y_recompute:
                self._pending_side = weight_grads
            else:
                self._side_wait_main()
                with torch.cuda.stream(self.side):
                    weight_grads()
        else:
            weight_grads()
        if dx0 is not None:
            S = 0
            if stats_target is not None and self.fuse_bn_stats and self.fuse_bn_bwd:
                S = ops.dwconv3x3_bwd_data_bnstats_slabs(view_in, n, h, w)
            if S > 0 and dwf:
                tb, C = stats_target, view_in.channels
                if bb.dwpart is None or bb.dwpart.numel() < S * 9 * C:
                    bb.dwpart = torch.empty(S * 9 * C, dtype=torch.float32, device=self.device)
                ops.dwconv3x3_bwd_data_bnstats_dwf(view_in, n, h, w, dk, dy, dx0, tb.mean if self.use_bn else None,
                                                   tb.rstd if self.use_bn else None, self._bnpart(tb, S, C),
                                                   bb.dwpart[:S * 9 * C])
                tb.bn_slabs = S
                self.run_beside(lambda: ops.reduce_slabs(bb.dwpart[:S * 9 * C], S, 9 * C, gdk))
            elif S > 0:
                tb = stats_target
                ops.dwconv3x3_bwd_data_bnstats(view_in, n, h, w, dk, dy, dx0, tb.mean if self.use_bn else None,
                                               tb.rstd if self.use_bn else None, self._bnpart(tb, S, view_in.channels))
                tb.bn_slabs = S
            else:
                ops.dwconv3x3_bwd_data(view_in, n, h, w, dk, dy, dx0, dx1)
        self._grads_ready(f"{b.name}_sepconv/depthwise_kernel")

    def _fused_bwd(self, b: Block, bb: BlockBufs, drop_rate: float = 0.0) -> bool:
        """The block's backward runs as one unet_sepconv_bwd_fused pass."""
        return self.fuse_block_bwd and self.fuse_bn_bwd and bb.y_recompute and drop_rate == 0.0 and b.cout == 64

    def _view_of(self, A: Acts, b: Block) -> View:
        bb = A.blocks[b.name]
        return View.bnrelu(bb.z, bb.scale, bb.shift)

    def backward(self, y_true: torch.Tensor, loss_kind: int = L.LOSS_DICE, loss_scale: float = 1.0) -> None:
        """Gradients of loss_scale x the loss of the last training forward into self.grads."""
        A = self._acts_last
        n = A.n
        seeds = self._last_seeds
        drop = seeds is not None and self.dropout_rate > 0.0
        last = self.dec[-1][4]
        hv, lb = self._view_of(A, last), A.blocks[last.name]
        S = (ops.head_bwd_bnstats_slabs(hv, n, self.h, self.w, self.num_classes)
             if self.fuse_bn_stats and self.fuse_bn_bwd else 0)
        if S > 0:  # the head's dx is all of the last block's da: emit its BN-backward partials too
            # binary head feeding the fused block backward: da = dlogit (x) kernel stays rank one
            # (one float per pixel stored instead of the 64-channel da, formed again on load)
            rank1 = self.num_classes == 1 and self._fused_bwd(last, lb)
            if rank1 and (lb.dlogit is None or lb.dlogit.numel() != n * self.h * self.w):
                lb.dlogit = torch.empty(n * self.h * self.w, dtype=torch.float32, device=self.device)
            ops.head_bwd_bnstats(hv, n, self.h, self.w, self.num_classes, self.vars["output_mask/kernel"], A.prob,
                                 y_true, A.sums, SMOOTH, loss_kind, None if rank1 else lb.da,
                                 self.gvars["output_mask/kernel"], self.gvars["output_mask/bias"],
                                 lb.mean if self.use_bn else None, lb.rstd if self.use_bn else None,
                                 self._bnpart(lb, S, hv.channels), loss_scale, dlogit=lb.dlogit if rank1 else None)
            lb.bn_slabs = S
            lb.da_rank1 = rank1
        else:
            ops.head_bwd(hv, n, self.h, self.w, self.num_classes, self.vars["output_mask/kernel"],
                         A.prob, y_true, A.sums, SMOOTH, loss_kind, lb.da,
                         self.gvars["output_mask/kernel"], self.gvars["output_mask/bias"], loss_scale)
        self._grads_ready("output_mask/kernel")
        nd = len(self.dec)
        for i in reversed(range(nd)):
            stage, fi, cin, b1, b2 = self.dec[i]
            self._block_bwd(A, b2, self._view_of(A, b1), A.blocks[b1.name].da, stats_target=A.blocks[b1.name])
            enc_b2 = self.enc[len(self.enc) - 1 - i][2]
            sk = A.blocks[enc_b2.name]
            vin = View.concat(A.up[stage], sk.z, sk.scale, sk.shift)
            if drop and i < nd - 1:
                vin = vin.dropout(self.dropout_rate, seeds[f"{stage}_dropout"])
            # skip half of the gradient is STORED into the encoder block's da (first contribution)
            self._block_bwd(A, b1, vin, A.dup[stage], sk.da)
            prev = self.dec[i - 1][4] if i > 0 else self.bneck[1]
            xv = self._view_of(A, prev)
            if i == 0 and drop:
                xv = xv.dropout(self.dropout_rate, seeds["bneck_dropout"])
            h, w = self._dims(b1.level + 1)
            gk, gb = self.gvars[f"{stage}_upsample/kernel"], self.gvars[f"{stage}_upsample/bias"]
            pb = A.blocks[prev.name]
            uk = self.vars[f"{stage}_upsample/kernel"]
            S = 0
            if self.fuse_bn_stats and self.fuse_bn_bwd:
                S = ops.conv_transpose2x2_bwd_data_bnstats_slabs(xv, n, h, w, fi)
            # data gradient on the critical path (emitting the BN partials of the block below when it
            # can), weight + bias gradients on the side stream
            if S > 0:
                ops.conv_transpose2x2_bwd_data_bnstats(xv, n, h, w, fi, uk, A.dup[stage], pb.da,
                                                       pb.mean if self.use_bn else None,
                                                       pb.rstd if self.use_bn else None, self._bnpart(pb, S, xv.c0),
                                                       kxt=self._ukt(stage))
                pb.bn_slabs = S
                pb.bn_masked = xv.drop_rate > 0.0  # (the bottleneck's dropout: the partials carry its mask)
            else:
                ops.conv_transpose2x2_bwd(xv, n, h, w, fi, uk, A.dup[stage], pb.da, None, None)
            if self.overlap:
                self._side_wait_main()
                with torch.cuda.stream(self.side):
                    ops.conv_transpose2x2_bwd(xv, n, h, w, fi, uk, A.dup[stage], None, gk, gb)
            else:
                ops.conv_transpose2x2_bwd(xv, n, h, w, fi, uk, A.dup[stage], None, gk, gb)
            self._grads_ready(f"{stage}_upsample/kernel")
        b1, b2 = self.bneck
        self._block_bwd(A, b2, self._view_of(A, b1), A.blocks[b1.name].da,
                        drop_rate=self.dropout_rate if drop else 0.0,
                        drop_seed=seeds["bneck_dropout"] if drop else 0, stats_target=A.blocks[b1.name])
        e4 = A.blocks[self.enc[-1][2].name]
        # pooled half ACCUMULATES into the encoder block's da (the skip half is already there)
        self._block_bwd(A, b1, View.pool_bnrelu(e4.z, e4.scale, e4.shift), e4.da, stats_target=e4,
                        view_f=View.bnrelu(e4.zsel, e4.scale, e4.shift))
        for j in reversed(range(len(self.enc))):
            stage, e1, e2 = self.enc[j]
            self._block_bwd(A, e2, self._view_of(A, e1), A.blocks[e1.name].da, stats_target=A.blocks[e1.name])
            if j > 0:
                pb = A.blocks[self.enc[j - 1][2].name]
                self._block_bwd(A, e1, View.pool_bnrelu(pb.z, pb.scale, pb.shift), pb.da, stats_target=pb,
                                view_f=View.bnrelu(pb.zsel, pb.scale, pb.shift))
            else:
                self._block_bwd(A, e1, View.plain(self._x_last), None)
        self._flush_side()
        if self.overlap:
            self._main_wait_side()

    # --------------------------------------------------------------- train step ------
    def forward_train(self, x: torch.Tensor, y_true: torch.Tensor) -> torch.Tensor:
        self.step_count += 1
        seeds = self.drop_seeds(self.step_count) if self.dropout_rate > 0 else None
        x = x.contiguous()
        self.forward(x, training=True, seeds=seeds)
        self._x_last = self._x_fwd
        self._acts_last = self.acts(x.shape[0])
        return self.loss(y_true.contiguous(), x.shape[0])

    def predict(self, x: torch.Tensor) -> torch.Tensor:
        """Inference forward (BN moving stats, no dropout); returns a new (N, H, W, ncls) tensor."""
        if self.graph_predict:
            return self._predict_graph(x)
        return self.forward(x, training=False).clone()

    def _predict_graph(self, x: torch.Tensor) -> torch.Tensor:
        """predict() through a HIP graph: per input shape (and routing attributes) the forward is
        run once eagerly on the graph's own stream -- every activation buffer and workspace is
        allocated there, outside the capture -- then captured; later calls copy x into the captured
        input and replay.  The graph reads the weights, moving statistics and split planes through
        their device pointers, so weight updates between calls are seen (the planes are re-split
        inside the graph, as the eager forward does)."""
        if x.dim() != 4 or tuple(x.shape[1:]) != (self.h, self.w, self.c):
            raise ValueError(f"expected input (N, {self.h}, {self.w}, {self.c}), got {tuple(x.shape)}")
        key = (tuple(x.shape), self.fuse_min_pixels, self.fuse_min_total, self.use_x3, self.params.data_ptr(),
               self.x3buf.data_ptr() if getattr(self, "x3buf", None) is not None else 0)
        ent = self._pgraphs.get(key)
        if ent is None:
            st = torch.cuda.Stream(device=self.device)  # one per graph: its workspace is never regrown
            xs = torch.empty(x.shape, dtype=torch.float32, device=self.device)
            st.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(st):
                xs.copy_(x)
                self.forward(xs, training=False)
            st.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                out = self.forward(xs, training=False)
            ent = self._pgraphs[key] = (g, xs, out, st)
        g, xs, out, _ = ent
        xs.copy_(x)
        g.replay()
        return out.clone()
