#!/bin/bash
# Fused separable-conv forward threshold re-checked with the register-A kernel: levels >= 64x64
# (default) vs >= 32x32 vs all levels (16x16).
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2 3; do
  for V in 4096 1024 256; do
    run ab_${V}_$i 300 env UNET_FUSE_MIN_HW=$V python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB fuse_min_hw=$V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab14.txt
  done
done
