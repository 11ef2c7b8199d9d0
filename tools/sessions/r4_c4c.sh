#!/bin/bash
# round 4: configs[4] per-GPU (21 classes, batch 8) bench and kernel trace with the final library
source "$(dirname "$0")/gpu_session.sh"
B4="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --num-classes 21 --batch 8"
run c4a 200 $B4
run c4tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4 -o c4 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
export UNET_OVERLAP=0
run c4s 200 $B4
