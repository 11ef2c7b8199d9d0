#!/bin/bash
# usage: tools/sessions/gpu_trace.sh TAG -- rocprofv3 kernel trace + stats of a short bench run (two-stream)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-tr}
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
