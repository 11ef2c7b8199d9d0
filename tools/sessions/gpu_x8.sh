#!/bin/bash
# Register-A fused forward with two stages of staging loads in flight (libunet_hip_deep.so):
# schedule-parity / sepconv op tests against it, encoder-block timings, step A/B.
source "$(dirname "$0")/gpu_session.sh"
L=unet-image-segmentation_amd/unet_amd
UNET_HIP_LIB=$L/libunet_hip_deep.so run t_sep 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "sepconv or schedule" --timeout 120 --timeout-method thread
run enc_base 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 32
UNET_HIP_LIB=$L/libunet_hip_deep.so run enc_deep 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 32
for i in 1 2; do
  for V in base deep; do
    case $V in base) E="UNET_X=0" ;; deep) E="UNET_HIP_LIB=$L/libunet_hip_deep.so" ;; esac
    run ab_${V}_$i 300 env $E python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB $V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab8.txt
  done
done
