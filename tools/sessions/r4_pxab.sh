#!/bin/bash
# round 4: the persistent forward on / off in the train step (lab library UNET_PX; UNET_PX_6464 for
# 64 -> 64 only), configs[1] alternated on one box, then a kernel trace of each
source "$(dirname "$0")/gpu_session.sh"
B1="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
for r in 1 2 3; do
  run px1_$r 200 env UNET_PX=1 $B1
  run px0_$r 200 env UNET_PX=0 $B1
  run px64off_$r 200 env UNET_PX=1 UNET_PX_6464=0 $B1
done
export UNET_PX=0
run tr0 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pxab -o px0 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0
export UNET_PX=1
run tr1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pxab -o px1 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0
