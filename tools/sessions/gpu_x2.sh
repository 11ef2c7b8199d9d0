#!/bin/bash
# Conv2DTranspose epilogue change: op tests + isolated timing; A/B of raised main-stream wave
# priority + deferred fused weight-gradient issue against the defaults.
source "$(dirname "$0")/gpu_session.sh"
L=unet-image-segmentation_amd/unet_amd
run t_convt 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "conv_transpose or convt" --timeout 120 --timeout-method thread
run convt 200 python tools/bench_convt.py
for i in 1 2; do
  for V in base pd; do
    case $V in
      base) E="UNET_X=0" ;; pd) E="UNET_SW_DEFER=1 UNET_HIP_LIB=$L/libunet_hip_prio.so" ;;
    esac
    run ab_${V}_$i 300 env $E python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB $V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab2.txt
  done
done
