#!/bin/bash
# Side-stream queue priority: low (default) vs the main stream's high priority.
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2 3; do
  for V in lo hi; do
    run ab_${V}_$i 300 env UNET_SIDE_PRIO=$V python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB side_prio=$V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab12.txt
  done
done
