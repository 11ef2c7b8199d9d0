#!/bin/bash
# new kernels' op tests first, then all GPU tests, then step A/Bs (split-precision forward, fused block backward)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3d}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "split_precision or pool_select or fused_sepconv or bwd_fused or pool_selection"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 400 python bench.py --no-cpu-baseline
run bench_nofb 300 python bench.py --no-cpu-baseline --encoder-batch 0 --no-fused-bwd
run bench_nox3 300 python bench.py --no-cpu-baseline --encoder-batch 0 --no-x3
run bench2 300 python bench.py --no-cpu-baseline --encoder-batch 0
