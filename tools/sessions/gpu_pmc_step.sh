#!/bin/bash
# usage: tools/sessions/gpu_pmc_step.sh TAG -- bench line + FETCH_SIZE / WRITE_SIZE passes of a short bench run (whole-step traffic)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-st}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
run bench 300 python bench.py --no-cpu-baseline --encoder-batch 0
run pmcF 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $B
run pmcW 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $B
