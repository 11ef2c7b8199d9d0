#!/bin/bash
# usage: tools/sessions/r6_bm.sh -- round 6: split-precision rows GEMM with 64-row tiles (three blocks per CU) on
# the short k-loops (K <= 128; lab UNET_X6_BM64_MAXK) vs 128-row tiles, per shape and in the step (lab library);
# and the 64-output blocks' fused block backward vs data-gradient GEMM + side-stream weight gradients (product)
source "$(dirname "$0")/gpu_session.sh"
LAB=$PWD/tools/labbin/libunet_hip_lab.so
run bm0 300 env UNET_HIP_LIB=$LAB UNET_X6_BM64_MAXK=0 python tools/bench_dgrad_x6.py bm128
run bm1 300 env UNET_HIP_LIB=$LAB UNET_X6_BM64_MAXK=128 python tools/bench_dgrad_x6.py bm64
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  run ab_bm1_$i 300 env UNET_HIP_LIB=$LAB UNET_X6_BM64_MAXK=128 $B
  run ab_bm0_$i 300 env UNET_HIP_LIB=$LAB UNET_X6_BM64_MAXK=0 $B
done
for i in 1 2; do
  run ab_fb1_$i 300 $B
  run ab_fb0_$i 300 $B --no-fused-bwd
done
