#!/bin/bash
# round 4: kernel trace of configs[4]'s per-GPU step (21 classes, batch 8), two streams and one
source "$(dirname "$0")/gpu_session.sh"
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8"
run tr 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o c4 -- $B
export UNET_OVERLAP=0
run tr1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o c4_1s -- $B
