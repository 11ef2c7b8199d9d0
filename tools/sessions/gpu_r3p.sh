#!/bin/bash
# two-blocks-per-CU filter-only weight-gradient kernel (64 / 128 outputs): op tests, parity, and the
# step A/B with the 128-output blocks recomputing y (bench --recompute-y128)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3p}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "bwd_filter or bwd_fused or sepconv_wgrad"
run model 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "train_step_parity"
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run a1 300 $B
run b1 300 $B --recompute-y128
run a2 300 $B
run b2 300 $B --recompute-y128
