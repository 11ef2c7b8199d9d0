#!/bin/bash
# deferred fused-backward slab reduction on the side stream (ABI 11): op tests, parity, same-box A/B
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3w}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "bwd_fused"
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
run model 600 python -u -m pytest tests/test_model_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run a1 300 $B
run p1 300 $B --no-defer-reduce
run a2 300 $B
run p2 300 $B --no-defer-reduce
