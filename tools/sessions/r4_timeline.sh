#!/bin/bash
# round 4: one-step HBM timeline: kernel trace (two streams), FETCH / WRITE
# passes and a single-stream trace of the SAME bench command; then the bench line of this build
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r4tl}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
run tr 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o ${TAG} -- $B
run pmcF 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tl -o ${TAG}_fetch -- $B
run pmcW 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tl -o ${TAG}_write -- $B
export UNET_OVERLAP=0
run tr1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o ${TAG}_1s -- $B
