#!/bin/bash
# round 4: depthwise filter-gradient grid 512 vs 1024 blocks (lab library UNET_DWF_BLOCKS),
# configs[4] per GPU (b8, 21 classes) and configs[1], alternated on one box
source "$(dirname "$0")/gpu_session.sh"
B4="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --num-classes 21 --batch 8"
B1="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
for r in 1 2 3; do
  run c4_d1024_$r 200 env UNET_DWF_BLOCKS=1024 $B4
  run c4_d512_$r 200 env UNET_DWF_BLOCKS=512 $B4
done
for r in 1 2; do
  run c1_d1024_$r 200 env UNET_DWF_BLOCKS=1024 $B1
  run c1_d512_$r 200 env UNET_DWF_BLOCKS=512 $B1
done
