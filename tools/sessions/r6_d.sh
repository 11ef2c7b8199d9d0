#!/bin/bash
# usage: tools/sessions/r6_d.sh -- round 6: split-precision fused forward with the depthwise taps in the
# halo pad floats (BN 128: 3 blocks per CU instead of 2).  Op tests + the training-geometry parity,
# then a same-box step A/B against the previous library (the lab build of the previous sources)
source "$(dirname "$0")/gpu_session.sh"
export UNET_PARITY_LOG=gpurun_out/parity_r6d.jsonl
run tests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_sizes_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread
OLD=tools/labbin/libunet_hip_lab.so
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  run ab_old_$i 300 env UNET_HIP_LIB=$OLD $B
  run ab_new_$i 300 $B
done
export N=16
S="python tools/sep_one.py 1 128 128 128 128 10 x3"
export UNET_HIP_LIB=$OLD
run kt_old 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6d -o old -- $S
unset UNET_HIP_LIB
run kt_new 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6d -o new -- $S
