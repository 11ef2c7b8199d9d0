#!/bin/bash
# round 4: weight-gradient GEMM with two stages of operand loads in flight (lab UNET_WGRAD_PD=2)
# vs one (1): isolated rows/wgrad shapes, then configs[1] step A/B on one box
source "$(dirname "$0")/gpu_session.sh"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
run iso1 300 env UNET_WGRAD_PD=1 python tools/bench_rows.py pd1
run iso2 300 env UNET_WGRAD_PD=2 python tools/bench_rows.py pd2
B1="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for r in 1 2 3; do
  run c1_pd1_$r 200 env UNET_WGRAD_PD=1 $B1
  run c1_pd2_$r 200 env UNET_WGRAD_PD=2 $B1
done
