#!/bin/bash
# usage: tools/sessions/gpu_ab_lib.sh ALT_SO -- bench A/B between the built libunet_hip.so and an alternative build
# of the same sources (e.g. a -D variant), swapping the file in place between runs (restored at the end).
source "$(dirname "$0")/gpu_session.sh"
L=unet-image-segmentation_amd/unet_amd
ALT=$1
cp $L/libunet_hip.so gpurun_out/base.so
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 0 ]; then cp $ALT $L/libunet_hip.so; else cp gpurun_out/base.so $L/libunet_hip.so; fi
  run bench_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
  grep -o '"value": [0-9.]*' gpurun_out/bench_$i.log | head -1
done
cp $ALT $L/libunet_hip.so
run ops 600 python -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -q -x
cp gpurun_out/base.so $L/libunet_hip.so
rm -f gpurun_out/base.so
