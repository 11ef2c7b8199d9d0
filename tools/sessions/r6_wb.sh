#!/bin/bash
# usage: tools/sessions/r6_wb.sh -- round 6: with the main stream now the step's critical path (x6 rows GEMMs), the
# side stream's weight-gradient grids at ~1 block per CU (UNET_WGRAD_BLOCKS 256 / 512) vs ~4 (1024, default);
# lab library, configs[1] step alternated
source "$(dirname "$0")/gpu_session.sh"
export UNET_HIP_LIB=$PWD/tools/labbin/libunet_hip_lab.so
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  run ab_wb1024_$i 300 $B
  run ab_wb512_$i 300 env UNET_WGRAD_BLOCKS=512 $B
  run ab_wb256_$i 300 env UNET_WGRAD_BLOCKS=256 $B
done
# the 128-output blocks' y recomputed by their (side-stream) weight-gradient pass instead of stored by the
# (critical-path) forward, product library
unset UNET_HIP_LIB
for i in 1 2; do
  run ab_ry0_$i 300 $B
  run ab_ry128_$i 300 $B --recompute-y128
  run ab_ry64128_$i 300 $B --recompute-y64-128
done
