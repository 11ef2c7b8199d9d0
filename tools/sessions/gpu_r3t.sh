#!/bin/bash
# XCD-contiguous slices of the fused / filter backward: op tests, parity, same-box A/B, step traffic
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3t}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "bwd_fused or bwd_filter"
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run a1 300 $B
run p1 300 env UNET_HIP_LIB=tools/lab/libunet_hip_prev.so $B
run a2 300 $B
run p2 300 env UNET_HIP_LIB=tools/lab/libunet_hip_prev.so $B
P="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
cp gpurun_out/a2.log gpurun_out/bench.log
run pmcF 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $P
run pmcW 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $P
