#!/bin/bash
# enc2_block1's depthwise filter gradient on the main stream's tail (UNET_TAIL_DWF=1): step A/B,
# model tests with it on.
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2 3; do
  for V in base tdwf; do
    case $V in base) E="UNET_X=0" ;; tdwf) E="UNET_TAIL_DWF=1" ;; esac
    run ab_${V}_$i 300 env $E python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB $V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab9.txt
  done
done
UNET_TAIL_DWF=1 run t_model 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread
