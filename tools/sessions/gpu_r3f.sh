#!/bin/bash
# A/B of a sepconv_rk change: its op tests, the step (default and without split precision), enc2_block1 alone
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3f}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "split_precision or pool_select or fused_sepconv or bwd_fused or pool_selection or sepconv"
run bench 400 python bench.py --no-cpu-baseline
run bench_nox3 300 python bench.py --no-cpu-baseline --encoder-batch 0 --no-x3
N=32 run e2b1 200 python tools/sep_one.py 1 128 128 64 128 10 x3
