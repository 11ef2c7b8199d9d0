#!/bin/bash
# round 4: rows-GEMM float4 C epilogue A/B (lab library, UNET_ROWS_F4=1 vs 0), then the rows GEMM
# GPU tests and a step A/B
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/lab/libunet_hip_lab.so
run f4_1 300 env UNET_HIP_LIB=$LAB UNET_ROWS_F4=1 python tools/bench_rows.py f4
run f4_0 300 env UNET_HIP_LIB=$LAB UNET_ROWS_F4=0 python tools/bench_rows.py dword
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_model_gpu.py
for i in 1 2; do
  for F in 1 0; do
    run st_${F}_$i 300 env UNET_HIP_LIB=$LAB UNET_ROWS_F4=$F python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB f4=$F $(grep -o '"value": [0-9.]*' gpurun_out/st_${F}_$i.log)" | tee -a gpurun_out/ab_f4.txt
  done
done
