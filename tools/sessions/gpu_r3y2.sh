#!/bin/bash
# round 3: kernel trace of the step with a sepconv_rk variant library (gaps around the fused forward)
source "$(dirname "$0")/gpu_session.sh"
export UNET_HIP_LIB=$PWD/tools/lab/librk_${1:-D}.so
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o rk${1:-D} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0
