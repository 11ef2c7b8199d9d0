#!/bin/bash
# XCD-aware block order (GEMM sibling grouping + contiguous depthwise / fused-forward tiles): op tests
# (same tiles, bitwise-equal results), parity, same-box A/B/C: all / GEMM grouping only / previous
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3r}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run opstests 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread
run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run a1 300 $B
run g1 300 env UNET_HIP_LIB=tools/lab/libunet_hip_g.so $B
run p1 300 env UNET_HIP_LIB=tools/lab/libunet_hip_prev.so $B
run a2 300 $B
run g2 300 env UNET_HIP_LIB=tools/lab/libunet_hip_g.so $B
run p2 300 env UNET_HIP_LIB=tools/lab/libunet_hip_prev.so $B
P="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
cp gpurun_out/a2.log gpurun_out/bench.log
run pmcF 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $P
run pmcW 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $P
