#!/bin/bash
# round 4: persistent split-precision sepconv forward -- lab (check + time vs the one-tile kernel,
# prefetch depth / blocks-per-CU variants through the lab library), then its GPU tests
source "$(dirname "$0")/gpu_session.sh"
run px_check 240 python tools/lab_px.py 32 both
LAB=tools/lab/libunet_hip_lab.so
run px_pd1 240 env UNET_HIP_LIB=$LAB UNET_PX_PD=1 python tools/lab_px.py 32 time
run px_pd2_b1 240 env UNET_HIP_LIB=$LAB UNET_PX_PD=2 UNET_PX_BPC=1 python tools/lab_px.py 32 time
run px_pd1_b1 240 env UNET_HIP_LIB=$LAB UNET_PX_PD=1 UNET_PX_BPC=1 python tools/lab_px.py 32 time
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_parity_sizes_gpu.py
