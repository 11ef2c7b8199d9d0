#!/bin/bash
# round 4: persistent sepconv forward after the scratch / race fixes + stream calibration
source "$(dirname "$0")/gpu_session.sh"
run px_check 240 python tools/lab_px.py 32 both
LAB=tools/lab/libunet_hip_lab.so
run px_pd1 240 env UNET_HIP_LIB=$LAB UNET_PX_PD=1 python tools/lab_px.py 32 time
run ko 300 tools/lab/x6_ko_lab 32
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "sepconv" 
run tests2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_parity_sizes_gpu.py
