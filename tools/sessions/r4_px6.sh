#!/bin/bash
# round 4: the persistent forward for 64 -> 64 too -- op/model tests, then configs[1] A/B with the
# lab library (UNET_PX_6464=0 keeps 64 -> 64 on the one-tile kernel)
source "$(dirname "$0")/gpu_session.sh"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run pxt 300 $T tests/test_ops_gpu.py -k "persistent or sepconv"
run model 500 $T tests/test_model_gpu.py tests/test_parity_sizes_gpu.py
B1="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
run a0 200 env UNET_PX_6464=0 $B1
run a1 200 env UNET_PX_6464=1 $B1
run b0 200 env UNET_PX_6464=0 $B1
run b1 200 env UNET_PX_6464=1 $B1
