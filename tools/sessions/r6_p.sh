#!/bin/bash
# usage: tools/sessions/r6_p.sh TAG -- round 6: kernel-trace stats of the configs[1] step (two-stream and single-stream)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r6p}
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0 --no-roofline
export UNET_OVERLAP=0
run prof1s 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_1s -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0
