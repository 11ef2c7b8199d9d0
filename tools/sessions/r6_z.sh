#!/bin/bash
# usage: tools/sessions/r6_z.sh -- round 6: split-precision fused forward, the stage's y stores left in flight across
# the weight-plane DMA wait (vmcnt(2)) vs waited for (vmcnt(0), tools/labbin/libunet_hip_base.so); configs[1] step
# with the encoder-block table at batch 32, alternated on one box
source "$(dirname "$0")/gpu_session.sh"
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 32"
for i in 1 2 3; do
  run ab_yw1_$i 300 $B
  run ab_yw0_$i 300 env UNET_HIP_LIB=$PWD/tools/labbin/libunet_hip_base.so $B
done
