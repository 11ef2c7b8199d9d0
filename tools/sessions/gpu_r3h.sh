#!/bin/bash
# Fused block backward in two-blocks-per-CU form: isolated timing, its op tests, the parity suite at
# the training geometry, the step
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3h}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run swko0 60 tools/lab/sw_fused_ko0
run opstests 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "bwd_fused or sepconv_bwd"
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
run bench 400 python bench.py --no-cpu-baseline --encoder-batch 0
