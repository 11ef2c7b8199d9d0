#!/bin/bash
# usage: tools/sessions/r6_w.sh -- round 6: split-precision weight-gradient GEMM (32-pixel stages, one LDS buffer):
# x6 tests, per-shape wgrad A/B and the configs[1] step A/B on the lab library (UNET_WGRAD_X6 = 0 / 1)
source "$(dirname "$0")/gpu_session.sh"
export UNET_HIP_LIB=$PWD/tools/labbin/libunet_hip_lab.so
run x6tests 300 env UNET_WGRAD_X6=1 python -u -m pytest tests/test_x6_gpu.py -x -q --timeout 120 --timeout-method thread
run wbench 300 python tools/bench_wgrad_x6.py wx6
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  run ab_w1_$i 300 env UNET_WGRAD_X6=1 $B
  run ab_w0_$i 300 env UNET_WGRAD_X6=0 $B
done
run ab_c4_w1 300 env UNET_WGRAD_X6=1 $B --num-classes 21 --batch 8
run ab_c4_w0 300 env UNET_WGRAD_X6=0 $B --num-classes 21 --batch 8
# the 64 x 64 level through the depthwise launch + the split-precision pointwise GEMM instead of the fused
# forward (engine.fuse_min_pixels / fuse_min_total), product library
unset UNET_HIP_LIB
for i in 1 2; do
  run ab_f64_$i 300 $B
  run ab_s64_$i 300 $B --fuse-min-pixels 16384 --fuse-min-total 1000000000
done
