#!/bin/bash
# split-precision fused forward: op tests first, then full GPU tests, bench with and without it
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3d}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "split_precision or pool_select or fused_sepconv"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 400 python bench.py --no-cpu-baseline
run bench_nox3 400 python bench.py --no-cpu-baseline --no-x3
run bench2 400 python bench.py --no-cpu-baseline --encoder-batch 0
