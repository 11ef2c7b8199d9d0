#!/bin/bash
# 256-column split-precision forward tile: its op tests, parity, same-box step A/B against the previous
# library (tools/lab/libunet_hip_prev.so), encoder table
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3k}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "split_precision or pool_selection or fused_sepconv"
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
run a1 300 python bench.py --no-cpu-baseline --encoder-batch 0
run b1 300 env UNET_HIP_LIB=tools/lab/libunet_hip_prev.so python bench.py --no-cpu-baseline --encoder-batch 0
run a2 300 python bench.py --no-cpu-baseline
run b2 300 env UNET_HIP_LIB=tools/lab/libunet_hip_prev.so python bench.py --no-cpu-baseline
