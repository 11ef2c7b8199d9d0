#!/bin/bash
# round 4: the narrow-N-tile rule's grid threshold 256 (default) vs 512 blocks (lab library knob
# UNET_ROWS_NARROW_MAX), configs[1] and configs[4] b8 alternated on one box
source "$(dirname "$0")/gpu_session.sh"
B1="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
B4="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
for r in 1 2 3; do
  run c1_256_$r 200 env UNET_ROWS_NARROW_MAX=256 $B1
  run c1_512_$r 200 env UNET_ROWS_NARROW_MAX=512 $B1
done
for r in 1 2; do
  run c4_256_$r 200 env UNET_ROWS_NARROW_MAX=256 $B4
  run c4_512_$r 200 env UNET_ROWS_NARROW_MAX=512 $B4
done
