#!/bin/bash
# usage: tools/sessions/r6_g.sh -- round 6: split-precision fused forward with the weight planes staged
# by LDS-DMA (global_load_lds_dwordx4 from inline asm, explicit vmcnt) instead of through registers.
# Op tests + training-geometry parity, a same-box step A/B against the previous product library
# (tools/labbin/libunet_hip_base.so), and kernel traces of the 64^2 blocks
source "$(dirname "$0")/gpu_session.sh"
export UNET_PARITY_LOG=gpurun_out/parity_r6g.jsonl
run tests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_sizes_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread
OLD=tools/labbin/libunet_hip_base.so
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  run ab_old_$i 300 env UNET_HIP_LIB=$OLD $B
  run ab_new_$i 300 $B
done
export N=16
for s in "1 64 64 128 256" "1 64 64 256 256" "1 128 128 64 128" "1 32 32 256 512"; do
  t=$(echo $s | tr ' ' _)
  S="python tools/sep_one.py $s 10 x3"
  export UNET_HIP_LIB=$OLD
  run kt_old_$t 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6g -o old_$t -- $S
  unset UNET_HIP_LIB
  run kt_new_$t 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6g -o new_$t -- $S
done
