#!/bin/bash
# Depthwise tiles of 8 channel quads x 32 columns (UNET_DW_QT=8) instead of 16 x 16 for C % 64 == 0:
# op tests with it, step A/B.
source "$(dirname "$0")/gpu_session.sh"
UNET_DW_QT=8 run t_dw 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "dwconv or bnstats" --timeout 120 --timeout-method thread
for i in 1 2 3; do
  for V in 16 8; do
    run ab_${V}_$i 300 env UNET_DW_QT=$V python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB dw_qt=$V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab13.txt
  done
done
