#!/bin/bash
# round 4: configs[4] per-GPU (21 classes, batch 8) bench, a kernel trace, and side-grid A/Bs at b8
# with the lab library (UNET_WGRAD_BLOCKS / UNET_DWF_BLOCKS)
source "$(dirname "$0")/gpu_session.sh"
B4="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --num-classes 21 --batch 8"
run c4a 200 $B4
run c4tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4 -o c4 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
run w1024 200 env UNET_WGRAD_BLOCKS=1024 $B4
run w512 200 env UNET_WGRAD_BLOCKS=512 $B4
run w256 200 env UNET_WGRAD_BLOCKS=256 $B4
run d512 200 env UNET_DWF_BLOCKS=512 $B4
run w1024b 200 env UNET_WGRAD_BLOCKS=1024 $B4
