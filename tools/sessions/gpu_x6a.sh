#!/bin/bash
# bf16x6 rows-GEMM A/B: microbench (fp32 product vs lab X6), step bench both ways, parity with X6
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/lab/libunet_hip_lab.so
run rows_f32 300 python tools/bench_rows.py f32
UNET_HIP_LIB=$LAB UNET_X6=1 run rows_x6 300 python tools/bench_rows.py x6
run bench_f32 300 python bench.py --no-cpu-baseline --encoder-batch 0
UNET_HIP_LIB=$LAB UNET_X6=1 run bench_x6 300 python bench.py --no-cpu-baseline --encoder-batch 0
UNET_HIP_LIB=$LAB UNET_X6=1 UNET_PARITY_LOG=gpurun_out/parity_x6.jsonl run parity_x6 600 python -u -m pytest tests/test_parity_sizes_gpu.py tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread
