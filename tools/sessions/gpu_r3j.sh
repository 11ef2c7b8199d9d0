#!/bin/bash
# rank-one head gradient (ABI 10): its op tests, all GPU tests, the step
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3j}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "head_bwd or bwd_fused"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 400 python bench.py --no-cpu-baseline --encoder-batch 0
run bench2 400 python bench.py --no-cpu-baseline --encoder-batch 0
run host 300 python tools/host_overhead.py
