#!/bin/bash
# fused block backward grid split (lab build, UNET_FB_SPLIT): same-box step A/B
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/lab/libunet_hip_lab2.so
B="python bench.py --no-cpu-baseline --encoder-batch 0"
for s in 1 4 2 8 1 4 2; do run s$s 300 env UNET_HIP_LIB=$LAB UNET_FB_SPLIT=$s $B; mv gpurun_out/s$s.log gpurun_out/s${s}_$RANDOM.log; done
