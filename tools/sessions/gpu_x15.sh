#!/bin/bash
# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the default: step A/B.
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2 3; do
  for V in 0 1; do
    run ab_${V}_$i 300 env HIP_FORCE_DEV_KERNARG=$V python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB dev_kernarg=$V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab15.txt
  done
done
