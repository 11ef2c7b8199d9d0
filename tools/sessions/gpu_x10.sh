#!/bin/bash
# Split-M weight-gradient grid re-checked with the round-2 defaults (wave priority 3, deferred fused
# weight gradient): 512 (2 blocks per CU, leaving registers for a main-stream wave) vs 1024.
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2; do
  for V in 1024 512 768; do
    run ab_${V}_$i 300 env UNET_WGRAD_BLOCKS=$V python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB wgrad_blocks=$V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab10.txt
  done
done
