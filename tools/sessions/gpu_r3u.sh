#!/bin/bash
# side-stream grid re-sweep after the XCD-aware orders (lab build knobs): weight-gradient GEMM blocks
# (UNET_WGRAD_BLOCKS, default 1024) and depthwise filter-gradient blocks (UNET_DWF_BLOCKS, default 1024)
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/lab/libunet_hip_lab2.so
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run d1 300 env UNET_HIP_LIB=$LAB $B
run w512 300 env UNET_HIP_LIB=$LAB UNET_WGRAD_BLOCKS=512 $B
run w2048 300 env UNET_HIP_LIB=$LAB UNET_WGRAD_BLOCKS=2048 $B
run f512 300 env UNET_HIP_LIB=$LAB UNET_DWF_BLOCKS=512 $B
run f2048 300 env UNET_HIP_LIB=$LAB UNET_DWF_BLOCKS=2048 $B
run d2 300 env UNET_HIP_LIB=$LAB $B
run w512b 300 env UNET_HIP_LIB=$LAB UNET_WGRAD_BLOCKS=512 $B
run f2048b 300 env UNET_HIP_LIB=$LAB UNET_DWF_BLOCKS=2048 $B
