#!/bin/bash
# split-K bottleneck GEMMs (ABI 11): op tests, parity, same-box step A/B (lab build, UNET_SPLITK=0/1)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3o}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "split_k or pointwise_bwd or conv_transpose"
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
LAB=tools/lab/libunet_hip_lab2.so
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run on1 300 env UNET_HIP_LIB=$LAB UNET_SPLITK=1 $B
run off1 300 env UNET_HIP_LIB=$LAB UNET_SPLITK=0 $B
run on2 300 env UNET_HIP_LIB=$LAB UNET_SPLITK=1 $B
run off2 300 env UNET_HIP_LIB=$LAB UNET_SPLITK=0 $B
run prod 300 $B
