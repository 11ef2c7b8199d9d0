#!/bin/bash
# usage: tools/sessions/gpu_pmc_bench.sh TAG -- clean single-stream kernel trace + FETCH_SIZE / WRITE_SIZE
# passes (separate runs, kernel-trace only) of a short bench.py run, for the roofline `traffic`.
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-run}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline"
export UNET_OVERLAP=0
run prof1s 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_1s -- $B
unset UNET_OVERLAP
run pmcF 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $B
run pmcW 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $B
