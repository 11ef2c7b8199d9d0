#!/bin/bash
# ABI 7 (unet_copy_strided in the image-block padding): op + model tests, bench.
source "$(dirname "$0")/gpu_session.sh"
run t_ops 600 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
run bench 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
