/*
 * unet_hip.h — C-ABI of libunet_hip.so, the MI355X (gfx950) engine for the
 * separable-conv U-Net hot path of planck-epoch/unet-image-segmentation.
 *
 * The reference has no native code and no FFI: every op on the path is an
 * implicit TensorFlow kernel emitted by a Keras layer.  Each entry point below
 * names the Keras layer / reference function it replaces (file:line in the
 * reference).  The reference-side binding a maintainer would add (ctypes) is
 * shown in INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - tensors are NHWC float32, dense (row stride = channel count), device
 *     memory owned by the caller; nothing here allocates device memory;
 *   - weights use the Keras layouts (see each function);
 *   - every call is asynchronous on `stream` (a hipStream_t; NULL = default);
 *   - return 0 on success, < 0 for an invalid argument, > 0 for a hipError_t;
 *     unet_last_error() gives a thread-local message for the last failure;
 *   - reductions are deterministic (fixed order, no float atomics): the same
 *     inputs give bitwise-identical outputs run to run;
 *   - ops needing scratch take (ws, ws_bytes); query the size with the
 *     matching *_workspace() function.
 */
#ifndef UNET_HIP_H
#define UNET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UNET_ABI_VERSION 12

typedef void* unet_stream_t; /* hipStream_t */

/* ---------------------------------------------------------------------------
 * Activation views.  Producers store raw (pre-BatchNorm) conv outputs; a
 * consumer reads the activation it needs through a view, which applies the
 * BatchNormalization affine + ReLU of model/u_net.py:22-25 on load, and
 * optionally MaxPooling2D (u_net.py:69), Concatenate (u_net.py:95-96) and
 * Dropout (u_net.py:77-78, 97-98).  The logical tensor is (n, h, w, c0 + c1).
 * ------------------------------------------------------------------------ */
enum {
    UNET_VIEW_PLAIN = 0,       /* x = src0                                    */
    UNET_VIEW_BNRELU = 1,      /* x = relu(src0 * scale0 + shift0)            */
    UNET_VIEW_POOL_BNRELU = 2, /* x = maxpool2x2(relu(src0*scale0+shift0)),
                                  src0 is (n, 2h, 2w, c0)                     */
    UNET_VIEW_CONCAT = 3       /* x = [src0 (raw, c0) | relu(src1*scale1+shift1) (c1)] */
};

typedef struct unet_view {
    int32_t mode;
    int32_t c0;
    int32_t c1;          /* CONCAT only, else 0 */
    int32_t reserved0;
    const float* src0;
    const float* scale0; /* per-channel, BNRELU / POOL_BNRELU */
    const float* shift0;
    const float* src1;   /* CONCAT: skip tensor (n, h, w, c1) */
    const float* scale1;
    const float* shift1;
    float drop_rate;     /* Dropout on the logical tensor; 0 = off */
    int32_t reserved1;
    uint64_t drop_seed;  /* keep(i) = u(splitmix64(seed + i*golden)) >= rate */
} unet_view;

int unet_abi_version(void);
const char* unet_last_error(void);

/* Cross-stream ordering for a caller that splits the backward over two HIP
 * streams of one device (the reference has no counterpart: TF schedules its
 * own graph).  The event carries no timing and only a device-scope release
 * (hipEventDisableSystemFence): ordering between the streams, not visibility
 * to the host.  unet_stream_wait_stream records `event` on `producer` and
 * makes `waiter` wait for it; the event can be reused at once.              */
int unet_event_create(void** event);
int unet_event_destroy(void* event);
int unet_stream_wait_stream(unet_stream_t waiter, unet_stream_t producer,
                            void* event);

/* Channel-strided copy: dst[r * dst_ld + c] = src[r * src_ld + c] for r < rows, c < cols.
 * The image block's 3 -> 4 channel zero padding (model/u_net.py:58 Input of 3 channels; the pad
 * channel of dst is left as it is) and the Keras-shaped (3, 3, 3, 1) / (1, 1, 3, 64) slices of
 * its padded kernels and their gradients, so no step copy goes through a framework kernel.   */
int unet_copy_strided(const float* src, int64_t rows, int cols, int64_t src_ld, float* dst,
                      int64_t dst_ld, unet_stream_t stream);

/* Split-precision weights: for each segment i (segs[4 i .. 4 i + 3] = source offset, rows,
 * cols, destination offset; host array, offsets in elements), dst + dst_off holds three bf16
 * planes [3][cols][rows] (transposed) with src[r][c] == hi + mid + lo exactly (round-to-nearest
 * bf16 of the value, then of each remainder).  One launch for every pointwise kernel of a step.
 * dst offsets must be multiples of 8 (16-B planes); rows * cols per plane.                  */
#define UNET_SPLIT_MAX_SEGS 64
int unet_split_x3(const float* src, const int64_t* segs, int nseg, unsigned short* dst,
                  unet_stream_t stream);
/* The same split with the planes in the source layout, [3][rows][cols] (ABI 12): the operand
 * layout of the split-precision data-gradient GEMM (unet_pointwise_bwd_data_bnrelu_x3 reads
 * pw_kernel (Cin, Cout) with k = Cout contiguous).                                            */
int unet_split_x3_keep(const float* src, const int64_t* segs, int nseg, unsigned short* dst,
                       unet_stream_t stream);
/* Both layouts in one launch: segs[5 i .. 5 i + 4] = source offset, rows, cols, destination
 * offset, keep (non-zero: [3][rows][cols], else [3][cols][rows]); the train step's one split per
 * weight update (ABI 12).                                                                      */
int unet_split_x3_mixed(const float* src, const int64_t* segs, int nseg, unsigned short* dst,
                        unet_stream_t stream);

/* Writes the logical tensor of a view, out (n, h, w, c0 + c1): the activation relu(bn(z)),
 * its max-pool, or the (dropped-out) concat.  The training path never needs this (consumers
 * read views directly); it serves eager conv_block outputs and inspection.                 */
int unet_view_materialize(const unet_view* x, int n, int h, int w, float* out,
                          unet_stream_t stream);

/* ----- SeparableConv2D(f, 3, padding='same') — model/u_net.py:14-20 --------
 * Depthwise half: y[n,h,w,c] = sum_{i,j<3} x[n,h+i-1,w+j-1,c] * k[i,j,c],
 * zero padding.  dw_kernel is Keras `depthwise_kernel` (3, 3, C, 1).       */
int unet_dwconv3x3_fwd(const unet_view* x, int n, int h, int w,
                       const float* dw_kernel, float* y, unet_stream_t stream);

/* Gradient w.r.t. the view's input.  Routing by view mode:
 *   PLAIN / BNRELU : dx0 (n,h,w,c0) = d(logical x)   (store)
 *   POOL_BNRELU    : dx0 (n,2h,2w,c0) += grad routed to the first max of each
 *                    2x2 window (accumulates: the skip path stored first)
 *   CONCAT         : dx0 (n,h,w,c0) = grad of the upsample half (store),
 *                    dx1 (n,h,w,c1) = grad of the skip half (store)
 * Dropout (if the view has it) is applied to the gradient first.          */
int unet_dwconv3x3_bwd_data(const unet_view* x, int n, int h, int w,
                            const float* dw_kernel, const float* dy,
                            float* dx0, float* dx1, unet_stream_t stream);
/* POOL_BNRELU view (the MaxPooling2D of u_net.py:69 feeding the next encoder
 * block) or BNRELU view (block1 -> block2 of a stage): unet_dwconv3x3_bwd_data
 * plus the BatchNorm-backward partial sums of the view's block, whose da this
 * launch completes (POOL: adds the pooled half of the gradient to the stored
 * skip half, reading the block's raw z for the argmax anyway; BNRELU: writes
 * all of da and reads z once for the ReLU mask): bn_partials[s][0][c] = sum g, [s][1][c] = sum g*xhat over
 * slab s, g = da*[z*scale+shift > 0], xhat = (z-mean)*rstd (mean/rstd NULL when
 * use_batch_norm=False).  Replaces unet_bn_relu_bwd_stats's pass over (da, z);
 * finish with unet_bn_relu_bwd_stats_finish.  _slabs returns the slab count S
 * (bn_partials holds S*2*C floats), 0 if the shape has no such path.          */
int unet_dwconv3x3_bwd_data_bnstats_slabs(const unet_view* x, int n, int h, int w);
/* (bn_partials: unet_bn_stats_partials_size(S, C) bytes, see the finish below) */
int unet_dwconv3x3_bwd_data_bnstats(const unet_view* x, int n, int h, int w,
                                    const float* dw_kernel, const float* dy,
                                    float* dx0, const float* mean,
                                    const float* rstd, float* bn_partials,
                                    unet_stream_t stream);
/* The same for a BNRELU view without dropout (round 6, ABI 12) that ALSO accumulates the
 * layer's depthwise FILTER gradient from the same registers (d_dw[t][c] = sum_q x[q] dy[q - off(t)],
 * x[q] = relu(z sc + sh) from the z the statistics read anyway): per tile a fixed-order [9][C]
 * slab into dw_partials ([S][9][C], S = _slabs(...)); unet_reduce_slabs(dw_partials, S, 9 C,
 * d_dw_kernel) sums them in tile order.  Replaces unet_dwconv3x3_bwd_filter's second pass over
 * dy and the view for such a block (model/u_net.py:14-20, the GradientTape's depthwise gradient). */
int unet_dwconv3x3_bwd_data_bnstats_dwf(const unet_view* x, int n, int h, int w,
                                        const float* dw_kernel, const float* dy, float* dx0,
                                        const float* mean, const float* rstd, float* bn_partials,
                                        float* dw_partials, unet_stream_t stream);
/* out[l] = sum_{s < S} slabs[s * len + l], summed in a fixed order (deterministic); slabs is
 * scratch (overwritten).  The reduction of unet_dwconv3x3_bwd_data_bnstats_dwf's slabs.        */
int unet_reduce_slabs(float* slabs, int S, int64_t len, float* out, unet_stream_t stream);

size_t unet_dwconv3x3_bwd_filter_workspace(int n, int h, int w, int c);
/* d_dw_kernel (3,3,C,1) = sum over pixels of x(shifted) * dy (overwrites). */
int unet_dwconv3x3_bwd_filter(const unet_view* x, int n, int h, int w,
                              const float* dy, float* d_dw_kernel,
                              void* ws, size_t ws_bytes, unet_stream_t stream);

/* Pointwise half: z[m, co] = sum_ci y[m, ci] * k[ci, co];  pw_kernel is Keras
 * `pointwise_kernel` (1, 1, Cin, Cout).  If bn_partials != NULL the epilogue
 * also writes per-tile BatchNorm statistics (count-weighted mean and M2 per
 * channel) for unet_bn_finalize.                                            */
size_t unet_bn_partials_size(int64_t m, int c); /* bytes of bn_partials */
int unet_pointwise_fwd(const float* y, int64_t m, int cin, int cout,
                       const float* pw_kernel, float* z, float* bn_partials,
                       unet_stream_t stream);
/* The same with pw_kernel_x3 = unet_split_x3(pw_kernel) ([3][Cout][Cin], unet_sepconv_fwd's planes;
 * ABI 12): the bf16x6 split-precision GEMM of unet_pointwise_bwd_data_bnrelu_x3 where cin % 32 == 0. */
int unet_pointwise_fwd_x3(const float* y, int64_t m, int cin, int cout, const float* pw_kernel,
                          const unsigned short* pw_kernel_x3, float* z, float* bn_partials,
                          unet_stream_t stream);
/* dy[m, ci] = sum_co dz[m, co] * k[ci, co] */
int unet_pointwise_bwd_data(const float* dz, int64_t m, int cin, int cout,
                            const float* pw_kernel, float* dy,
                            unet_stream_t stream);
size_t unet_pointwise_bwd_filter_workspace(int64_t m, int cin, int cout);
/* d_pw_kernel[ci, co] = sum_m y[m, ci] * dz[m, co] (overwrites) */
int unet_pointwise_bwd_filter(const float* y, const float* dz, int64_t m,
                              int cin, int cout, float* d_pw_kernel,
                              void* ws, size_t ws_bytes, unet_stream_t stream);
/* Fused SeparableConv2D: depthwise 3x3 of the view -> pointwise 1x1 (+ BatchNorm partials as
 * unet_pointwise_fwd), the depthwise result never leaving the chip except as the optional `y`
 * (needed by the pointwise weight gradient in training; NULL for inference).  Supported when
 * unet_sepconv_fwd_supported() says so (h % 8 == 0, w % 16 == 0, channels % 4 == 0).     */
int unet_sepconv_fwd_supported(const unet_view* x, int n, int h, int w, int cout);
int unet_sepconv_fwd(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                     int cout, const float* pw_kernel,
                     const unsigned short* pw_kernel_x3, float* y, float* z,
                     float* bn_partials, float* z_pool_sel, const float* gamma,
                     unet_stream_t stream);
/* pw_kernel_x3 (optional): pw_kernel split by unet_split_x3 ([3][Cout][Cin] bf16 planes).  With
 * it the register-A kernel runs its split-precision MFMA variant where it exists (channels
 * % 16 == 0, no max-pool view): every product of the pointwise GEMM is formed from the three
 * bf16 parts of both operands, x == hi + mid + lo exactly, and summed as the six significant
 * part products on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (error ~2^-23 |a b| per
 * product, below fp32 accumulation rounding: DESIGN.md "Split-precision MFMA").              */
/* z_pool_sel (optional, (N, h/2, w/2, cout)): the encoder stage's MaxPooling2D((2,2))
 * (model/u_net.py:69) prepared for its consumer: per 2x2 window of z and channel, the raw
 * value the max-pool of relu(z * scale + shift) selects -- the window max where gamma >= 0,
 * the min where gamma < 0 (gamma = the block's BN gamma; NULL = no BatchNorm: max).  scale has
 * gamma's sign and fmaf / relu are monotone, so a BNRELU view of z_pool_sel reads exactly the
 * pooled activation, one value per output pixel instead of four.  Written by the kernel's
 * epilogue (register-A schedule) or by unet_pool_select after it.  The max-pool BACKWARD still
 * routes through z (first maximum of the window): POOL_BNRELU views of z.                   */
int unet_pool_select(const float* z, int n, int h, int w, int c, const float* gamma,
                     float* out, unet_stream_t stream);
/* Kernel schedule of unet_sepconv_fwd (process-wide; returns the previous value, < 0 on a bad
 * value).  AUTO: the register-A kernel (each lane computes the depthwise output straight in the
 * MFMA operand layout) for BN+ReLU / concat / plain views of >= 64 input and output channels
 * and for max-pool views of >= 64 inputs and 64..128 outputs; the LDS-A-tile kernel otherwise
 * (max-pool views of > 128 outputs: its 256-wide tile pools each halo element once for all
 * columns).  TILE / RK force one (RK fails with -1 where it does not exist): both are
 * parity-tested (tests/test_ops_gpu.py).  With pw_kernel_x3, 64 / 128 input and output channels and
 * a plain / BN+ReLU / concat view, RK runs the register-A kernel PERSISTENT over pixel tiles
 * (sepconv_px.hip: a block walks a run of tiles as one stream of k-stages, the next stages' loads
 * in flight across tile boundaries); AUTO does so only where that measured faster inside the train
 * step (128 outputs from 64 inputs or with z_pool_sel); RK1 forces the one-tile-per-block
 * register-A kernel (same products, same per-tile statistics partials up to the order of the
 * 4-wave combine).
 * Without pw_kernel_x3 the results are identical: both
 * form each output as the same k-ordered fmaf chain.  With pw_kernel_x3 the register-A kernel
 * runs its split-precision (bf16x6 MFMA) variant, whose summation order differs (results within
 * fp32 rounding, not bitwise), while TILE ignores the split planes and gives the fmaf-chain
 * results: the output then depends on the schedule.                                          */
enum { UNET_SEPCONV_AUTO = 0, UNET_SEPCONV_TILE = 1, UNET_SEPCONV_RK = 2, UNET_SEPCONV_RK1 = 3 };
int unet_sepconv_set_schedule(int schedule);

/* Both weight gradients of a SeparableConv2D (model/u_net.py:14-20; the pixel reductions of
 * Keras' implicit backward, scripts/train.py:308) in one pass WITHOUT the depthwise output y:
 *   d_pw_kernel[ci, co] = sum_m y[m, ci] * dz[m, co],  y = depthwise3x3(view x) recomputed
 *   d_dw_kernel[t, ci]  = sum_m x[m + off(t), ci] * dy[m, ci]
 * so the training forward need not store y (unet_sepconv_fwd with y = NULL).  Replaces
 * unet_pointwise_bwd_filter over a stored y + unet_dwconv3x3_bwd_filter; both overwritten.
 * Supported (unet_sepconv_bwd_filter_supported) for the HBM-bound 64-output blocks of the
 * widest level: input channels % 64 == 0, 64 output channels, PLAIN / BNRELU / CONCAT view,
 * h % 8 == 0, w % 16 == 0; dy / dz / the depthwise kernel / view sources 16-B aligned.       */
int unet_sepconv_bwd_filter_supported(const unet_view* x, int n, int h, int w, int cout);
size_t unet_sepconv_bwd_filter_workspace(int n, int h, int w, int cin, int cout);
int unet_sepconv_bwd_filter(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                            const float* dy, const float* dz, int cout, float* d_dw_kernel,
                            float* d_pw_kernel, void* ws, size_t ws_bytes, unet_stream_t stream);
/* The same pass for a 64-output block ALSO doing the block's BatchNorm + ReLU backward and
 * pointwise data gradient (model/u_net.py:14-25, the GradientTape of scripts/train.py:308): per
 * pixel tile dz = scale (g - p - (z - mu) q), g = da [z scale + shift > 0] with coef = (mu, p, q)
 * from unet_bn_relu_bwd_stats(_finish) (exactly unet_pointwise_bwd_data_bnrelu's dz), then
 * dy = dz . pw_kernel^T (written out, for the depthwise data gradient), d_pw_kernel = y^T dz and
 * d_dw_kernel as above; dz never goes to memory (bytes: da, z, the input view, dy).  No dropout
 * on either side.  Workspace as unet_sepconv_bwd_filter.
 * da may be NULL when da_dlogit (m floats) and da_kernel (cout floats) are given: the binary
 * head's gradient is rank one, da[m][c] = da_dlogit[m] * da_kernel[c] (unet_head_bwd_bnstats'
 * dlogit output and the head's 1x1 kernel, model/u_net.py:105-112), formed on load with the
 * same product the head would have stored (ABI 10).                                          */
int unet_sepconv_bwd_fused(const unet_view* x, int n, int h, int w, const float* dw_kernel,
                           const float* pw_kernel, const float* da, const float* da_dlogit,
                           const float* da_kernel, const float* z,
                           const float* scale, const float* shift, const float* coef, int cout,
                           float* dy, float* d_dw_kernel, float* d_pw_kernel, void* ws,
                           size_t ws_bytes, unet_stream_t stream);

/* ----- BatchNormalization() — model/u_net.py:22-23 (Keras defaults:
 * momentum 0.99, epsilon 1e-3, biased batch variance for both the output
 * and the moving-variance update).  Training: reduces bn_partials into the
 * batch mean / variance, writes mean, rstd = 1/sqrt(var+eps), and the affine
 * scale = gamma*rstd, shift = beta - mean*scale consumed by views; updates
 * moving stats when update_moving != 0.  gamma == NULL means
 * use_batch_norm=False: scale = 1, shift = beta (the sepconv bias).
 * One launch: 64-partial chunk sums, then the last block of each 64-channel
 * column to finish sums the chunk rows.  The tail of bn_partials (past the
 * per-tile partials) holds the chunk rows and ceil(c/64) arrival counters:
 * the buffer must hold unet_bn_partials_size bytes and its counters must be
 * zero before the first call (allocate it zeroed once; calls leave them
 * zero; the statistics producers never write past the per-tile partials).   */
int unet_bn_finalize(float* bn_partials, int64_t m, int c,
                     const float* gamma, const float* beta, float eps,
                     float momentum, float* moving_mean, float* moving_var,
                     int update_moving, float* mean, float* rstd,
                     float* scale, float* shift, unet_stream_t stream);
/* SyncBN under data parallelism (SURVEY §8(e) option; off by default: the reference's
 * tf.distribute default, and Keras BatchNormalization(synchronized=False), normalise each
 * replica over its own shard).  unet_bn_moments reduces this replica's partials (as
 * unet_bn_finalize does, same counters) to a record of 1 + 2c doubles: (count, mean[c], M2[c]);
 * the caller gathers the replicas' records ([world][1 + 2c], rank order) and
 * unet_bn_finalize_moments combines them in rank order (Chan's parallel formula, double) and
 * finalizes exactly as unet_bn_finalize with the global-batch mean / biased variance.  Every
 * replica combining the same gathered records ends with identical statistics.
 * Backward: unet_bn_bwd_coef forms coef = (mean, S1/m, rstd*S2/m) from the all-reduced sums
 * sums[0..c) = sum g, sums[c..2c) = sum g*xhat over all replicas (m = the global pixel count);
 * the replica's own dgamma / dbeta stay its local sums (the gradient all-reduce averages them). */
int unet_bn_moments(float* bn_partials, int64_t m, int c, double* moments, unet_stream_t stream);
int unet_bn_finalize_moments(const double* moments, int world, int c, const float* gamma,
                             const float* beta, float eps, float momentum, float* moving_mean,
                             float* moving_var, int update_moving, float* mean, float* rstd,
                             float* scale, float* shift, unet_stream_t stream);
int unet_bn_bwd_coef(const float* sums, int64_t m, int c, int use_bn, const float* mean,
                     const float* rstd, float* coef, unet_stream_t stream);

/* Inference: scale/shift from the moving statistics. */
int unet_bn_infer_params(const float* gamma, const float* beta,
                         const float* moving_mean, const float* moving_var,
                         int c, float eps, float* scale, float* shift,
                         unet_stream_t stream);
/* Backward of a = dropout(relu(z*scale+shift)):
 *   g = da * keep/(1-rate) * [z*scale+shift > 0]
 *   dbeta = sum g, dgamma = sum g*xhat (xhat = (z-mean)*rstd)
 *   dz = scale*(g - dbeta/M - xhat*dgamma/M)    (use_bn != 0)
 *   dz = g, dbeta = sum g, dgamma untouched       (use_bn == 0, bias grad)  */
size_t unet_bn_relu_bwd_workspace(int64_t m, int c);
int unet_bn_relu_bwd(const float* da, const float* z, int64_t m, int c,
                     const float* mean, const float* rstd, const float* scale,
                     const float* shift, int use_bn, float drop_rate,
                     uint64_t drop_seed, float* dgamma, float* dbeta,
                     float* dz, void* ws, size_t ws_bytes,
                     unet_stream_t stream);
/* Statistics half of unet_bn_relu_bwd (same workspace): dgamma / dbeta and the
 * per-channel coefficients coef[3c] = (mean, dbeta/M, rstd*dgamma/M) (zeros when
 * use_bn == 0) with which unet_pointwise_bwd_data_bnrelu forms dz on load, so dz
 * never takes a separate HBM pass.  Same reference lines as unet_bn_relu_bwd.     */
int unet_bn_relu_bwd_stats(const float* da, const float* z, int64_t m, int c,
                           const float* mean, const float* rstd,
                           const float* scale, const float* shift, int use_bn,
                           float drop_rate, uint64_t drop_seed, float* dgamma,
                           float* dbeta, float* coef, void* ws, size_t ws_bytes,
                           unet_stream_t stream);
/* Finish of the statistics from S producer-side partial slabs ([S][2][c],
 * fixed-order double reduction): the outputs of unet_bn_relu_bwd_stats, in one
 * launch (64-slab chunk sums; the last block of each channel range to finish
 * sums the chunk rows).  The partials buffer holds
 * unet_bn_stats_partials_size(S, c) bytes: the slabs, the chunk rows, then
 * ceil(c/64) arrival counters that must be zero before the first call --
 * allocate the buffer zeroed once; every call leaves them zero again.        */
size_t unet_bn_stats_partials_size(int S, int c);
int unet_bn_relu_bwd_stats_finish(float* partials, int S, int64_t m, int c,
                                  const float* mean, const float* rstd,
                                  int use_bn, float* dgamma, float* dbeta,
                                  float* coef, unet_stream_t stream);
/* Pointwise data gradient of a conv_block whose output went through BN + ReLU
 * (+ dropout): dz = scale*(g - coef_p - (z - coef_mu)*coef_q),
 * g = da * keep/(1-rate) * [z*scale+shift > 0], is formed while loading the GEMM
 * operand; dy[m, ci] = sum_co dz[m, co] * k[ci, co].  If dz != NULL the formed dz
 * is also stored (the pointwise weight gradient reads it).  cin, cout % 4 == 0.
 * Replaces the backward of model/u_net.py:20-25 (SeparableConv2D pointwise ->
 * BatchNormalization -> ReLU) for the data path.                                 */
int unet_pointwise_bwd_data_bnrelu(const float* da, const float* z, int64_t m,
                                   int cin, int cout, const float* pw_kernel,
                                   const float* scale, const float* shift,
                                   const float* coef, float drop_rate,
                                   uint64_t drop_seed, float* dy, float* dz,
                                   unet_stream_t stream);
/* The same with pw_kernel_x3 = unet_split_x3_keep(pw_kernel) ([3][Cin][Cout] bf16 planes, 16-B
 * aligned; ABI 12): where cout % 32 == 0 the GEMM runs the six significant bf16 part products
 * of both operands on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the A operand, dz, is
 * split exactly as it is formed), the split-precision form of unet_sepconv_fwd's pw_kernel_x3:
 * fp32-accurate (relative error ~2^-23 per product), not bitwise equal to the fp32-MFMA route.
 * pw_kernel is still read where the route does not apply.                                   */
int unet_pointwise_bwd_data_bnrelu_x3(const float* da, const float* z, int64_t m,
                                      int cin, int cout, const float* pw_kernel,
                                      const unsigned short* pw_kernel_x3,
                                      const float* scale, const float* shift,
                                      const float* coef, float drop_rate,
                                      uint64_t drop_seed, float* dy, float* dz,
                                      unet_stream_t stream);

/* The image block (enc1_block1 over the 3-channel input zero-padded to 4):
 * unet_pointwise_bwd_data_bnrelu without dropout, cin == 4, cout 32 or 64,
 * that also writes the pointwise kernel gradient d_pw_kernel[ci][co] =
 * sum_m y[m,ci] dz[m,co] (y: the depthwise output, m x 4) from the dz it forms
 * on load, so dz is never stored (one streaming pass over da, z, y).
 * Workspace: _workspace(m, cin, cout) bytes (0: shape not supported).      */
size_t unet_pointwise_bwd_data_bnrelu_wgrad_workspace(int64_t m, int cin,
                                                      int cout);
int unet_pointwise_bwd_data_bnrelu_wgrad(const float* da, const float* z,
                                         int64_t m, int cin, int cout,
                                         const float* pw_kernel,
                                         const float* scale, const float* shift,
                                         const float* coef, const float* y,
                                         float* dy, float* d_pw_kernel,
                                         void* ws, size_t ws_bytes,
                                         unet_stream_t stream);

/* The image block's two weight gradients in ONE streaming pass (its data gradient is
 * never needed): as unet_pointwise_bwd_data_bnrelu_wgrad, but the dy it forms per
 * pixel is not stored, it is contracted at once with the pixel's 3x3 neighbourhood
 * of x into the depthwise kernel gradient.  x: the (n, h, w, 4) input the forward
 * read (channels past wcin zero), pw_kernel (4, cout) padded the same way.  Outputs
 * in the Keras shapes of the wcin-channel layer: d_dw_kernel (3, 3, wcin, 1),
 * d_pw_kernel (1, 1, wcin, cout) -- both overwritten.  cout 32 or 64.
 * Replaces the backward of the first SeparableConv2D (model/u_net.py:14-20 for
 * the first conv_block, u_net.py:62) for its weights.
 * Workspace: _workspace(n, h, w, cout) bytes (0: shape not supported).       */
size_t unet_image_block_bwd_wgrad_workspace(int n, int h, int w, int cout);
int unet_image_block_bwd_wgrad(const float* x, int n, int h, int w, int wcin,
                               int cout, const float* pw_kernel,
                               const float* scale, const float* shift,
                               const float* coef, const float* da,
                               const float* z, const float* y,
                               float* d_dw_kernel, float* d_pw_kernel,
                               void* ws, size_t ws_bytes,
                               unet_stream_t stream);

/* ----- Conv2DTranspose(f, 2, strides=2, padding='same') — u_net.py:88-94 --
 * out[n, 2i+a, 2j+b, co] = bias[co] + sum_ci x[n,i,j,ci] * k[a,b,co,ci];
 * kernel is Keras (2, 2, Cout, Cin), x a view of (n, h, w, Cin).           */
int unet_conv_transpose2x2_fwd(const unet_view* x, int n, int h, int w,
                               int cout, const float* kernel,
                               const float* bias, float* out,
                               unet_stream_t stream);
/* The same with kernel_x3 = unet_split_x3_keep(kernel as (4 cout, cin)) (ABI 12): the bf16x6
 * split-precision GEMM of unet_pointwise_bwd_data_bnrelu_x3 where cin % 32 == 0.            */
int unet_conv_transpose2x2_fwd_x3(const unet_view* x, int n, int h, int w, int cout,
                                  const float* kernel, const unsigned short* kernel_x3,
                                  const float* bias, float* out, unet_stream_t stream);
size_t unet_conv_transpose2x2_bwd_workspace(int n, int h, int w, int cin,
                                            int cout);
/* dx (n,h,w,Cin) = grad w.r.t. the view output (NULL: skip); dkernel, dbias
 * overwrite (both NULL: data gradient only, so the weight gradient can be a
 * separate call with dx = NULL, e.g. on another stream). */
int unet_conv_transpose2x2_bwd(const unet_view* x, int n, int h, int w,
                               int cout, const float* kernel,
                               const float* dout, float* dx, float* dkernel,
                               float* dbias, void* ws, size_t ws_bytes,
                               unet_stream_t stream);
/* Data gradient only, for a BNRELU view (the decoder block2 / bottleneck
 * output feeding the upsample, u_net.py:88): dx is then the whole da of the
 * view's block, so the GEMM epilogue also emits that block's BatchNorm-backward
 * partials in the unet_dwconv3x3_bwd_data_bnstats format (S = _slabs(...)
 * slabs, one per row tile: 128 rows, or 64 rows when the 128-row grid would
 * hold <= 256 tiles of 64 columns (round 5); always size and finish with the
 * S the query returns; mean/rstd NULL when use_batch_norm=False; finish with
 * unet_bn_relu_bwd_stats_finish).  Replaces unet_bn_relu_bwd_stats's separate
 * pass over (da, z).  A view with dropout (the bottleneck's, u_net.py:77-78;
 * round 5, no signature change): the partials are those of g = da * mask, as
 * unet_bn_relu_bwd_stats(..., drop_rate, drop_seed, ...) forms them; dx stays
 * the gradient w.r.t. the dropout output.  _slabs: 0 if the view or shape has
 * no such path.                                                              */
int unet_conv_transpose2x2_bwd_data_bnstats_slabs(const unet_view* x, int n,
                                                  int h, int w, int cout);
int unet_conv_transpose2x2_bwd_data_bnstats(const unet_view* x, int n, int h,
                                            int w, int cout,
                                            const float* kernel,
                                            const float* dout, float* dx,
                                            const float* mean,
                                            const float* rstd,
                                            float* bn_partials,
                                            unet_stream_t stream);
/* The same with kernel_x3t = unet_split_x3(kernel as (4 cout, cin)) ([3][cin][4 cout] planes,
 * ABI 12): the bf16x6 GEMM where cout % 8 == 0 and the partials are per 128-row tile.      */
int unet_conv_transpose2x2_bwd_data_bnstats_x3(const unet_view* x, int n, int h, int w, int cout,
                                               const float* kernel, const unsigned short* kernel_x3t,
                                               const float* dout, float* dx, const float* mean,
                                               const float* rstd, float* bn_partials,
                                               unet_stream_t stream);

/* ----- Output layer Conv2D(ncls, 1, activation) — u_net.py:105-112 --------
 * prob = sigmoid(x.k + b) (ncls == 1) or softmax over channels.            */
int unet_head_fwd(const unet_view* x, int n, int h, int w, int ncls,
                  const float* kernel, const float* bias, float* prob,
                  unet_stream_t stream);

/* ----- dice_coef / iou_coef / dice_loss — utils/metrics.py:6-62,
 * utils/loss.py:9-48.  Per (batch, channel) sums over H, W:
 * sums[b][c] = {sum t*p, sum t, sum p};  result = {1 - mean dice,
 * mean dice, mean iou}.  smooth = K.epsilon() = 1e-7 in the reference.     */
enum { UNET_LOSS_DICE = 0, UNET_LOSS_IOU = 1 };
size_t unet_dice_workspace(int n, int64_t hw, int ncls);
int unet_dice_fwd(const float* y_true, const float* y_pred, int n,
                  int64_t hw, int ncls, float smooth, float* sums,
                  float* result, void* ws, size_t ws_bytes,
                  unet_stream_t stream);
/* Backward of (1 - mean dice) [or 1 - mean iou] through the head
 * activation and the 1x1 conv: dx (n,h,w,Cin) grad w.r.t. the head input
 * view; dkernel (1,1,Cin,ncls), dbias (ncls) overwrite.  loss_scale (> 0)
 * multiplies the loss gradient: 1 for the reference's single-process step;
 * n_local * world / n_global for a data-parallel shard, so that the summed
 * all-reduce times 1/world is the gradient of the global-batch mean.       */
size_t unet_head_bwd_workspace(int n, int h, int w, int cin, int ncls);
int unet_head_bwd(const unet_view* x, int n, int h, int w, int ncls,
                  const float* kernel, const float* prob,
                  const float* y_true, const float* sums, float smooth,
                  int loss_kind, float loss_scale, float* dx, float* dkernel,
                  float* dbias,
                  void* ws, size_t ws_bytes, unet_stream_t stream);
/* Head on a BNRELU view (binary; or multi-class with <= 24 classes and
 * Cin in {4, 8, 16, 32, 64}, one fused pass; other multi-class shapes: the
 * _slabs query returns 0 and the call is refused -- use unet_head_bwd plus
 * unet_bn_relu_bwd_stats): unet_head_bwd plus the BatchNorm-backward
 * partial sums of the head input's block (dx is all of its da; bn_partials
 * layout and finish as unet_dwconv3x3_bwd_data_bnstats).  _slabs: S, or 0.
 * Binary only: dx may be NULL when dlogit (m floats) is given: dx = dlogit
 * (x) kernel is rank one, so only dL/dlogit per pixel is stored and the
 * consumer forms dx on load (unet_sepconv_bwd_fused's da_dlogit; ABI 10).   */
int unet_head_bwd_bnstats_slabs(const unet_view* x, int n, int h, int w, int ncls);
int unet_head_bwd_bnstats(const unet_view* x, int n, int h, int w, int ncls,
                          const float* kernel, const float* prob,
                          const float* y_true, const float* sums, float smooth,
                          int loss_kind, float loss_scale, float* dx,
                          float* dlogit, float* dkernel, float* dbias,
                          const float* mean, const float* rstd,
                          float* bn_partials, void* ws, size_t ws_bytes,
                          unet_stream_t stream);

/* ----- keras.metrics.MeanIoU(num_classes) — scripts/train.py:231,
 * scripts/benchmark.py:237,269.  Confusion counts (rows = true, cols =
 * pred) accumulate into `confusion` (num_classes^2 uint64).  threshold < 0:
 * Keras cast semantics (float -> int64 truncation, as in training on raw
 * probabilities); threshold >= 0: pred = (p > threshold) (benchmark.py:260).
 * Labels outside [0, num_classes) are skipped.                             */
int unet_meaniou_update(const float* y_true, const float* y_pred,
                        int64_t count, int num_classes, float threshold,
                        uint64_t* confusion, unet_stream_t stream);

/* ----- keras.optimizers.AdamW — scripts/train.py:226 (Keras 3 update):
 *   p -= p*wd*lr;  g *= grad_scale;  m += (g-m)(1-b1);  v += (g^2-v)(1-b2);
 *   p -= m*alpha / (sqrt(v) + eps),  alpha = lr*sqrt(1-b2^t)/(1-b1^t).      */
int unet_adamw_step(float* param, const float* grad, float* m, float* v,
                    int64_t count, float lr, float weight_decay, float beta1,
                    float beta2, float eps, float alpha, float grad_scale,
                    unet_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UNET_HIP_H */
