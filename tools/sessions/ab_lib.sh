#!/bin/bash
# usage: tools/sessions/ab_lib.sh N -- alternate the in-tree library and libunet_hip_ab.so, N benches each
source "$(dirname "$0")/gpu_session.sh"
AB=unet-image-segmentation_amd/unet_amd/libunet_hip_ab.so
for i in $(seq 1 "$1"); do
  for E in "UNET_X=$i" "UNET_HIP_LIB=$AB"; do
    run bench 300 env "$E" python bench.py --steps 30 --warmup 5 --no-cpu-baseline --encoder-batch 0
    echo "AB $E $(grep -o '"value": [0-9.]*' gpurun_out/bench.log)"
  done
done
