#!/bin/bash
# usage: tools/sessions/r6_c.sh TAG -- round 6: the persistent split-precision forward (sepconv_px) with
# 4 stages of loads in flight (lab UNET_PX_PD=4) and on every 64 / 128-channel shape (UNET_PX_ALL=1):
# isolated per-shape times and bitwise checks (tools/lab_px.py at batch 16), then a same-box step A/B
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/labbin/libunet_hip_lab.so
run px_pd2 300 env UNET_HIP_LIB=$LAB UNET_PX_PD=2 python tools/lab_px.py 16 both
run px_pd4 300 env UNET_HIP_LIB=$LAB UNET_PX_PD=4 python tools/lab_px.py 16 both
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  run ab_base_$i 300 env UNET_HIP_LIB=$LAB $B
  run ab_pd4_$i 300 env UNET_HIP_LIB=$LAB UNET_PX_PD=4 $B
  run ab_all2_$i 300 env UNET_HIP_LIB=$LAB UNET_PX_ALL=1 $B
  run ab_all4_$i 300 env UNET_HIP_LIB=$LAB UNET_PX_ALL=1 UNET_PX_PD=4 $B
done
