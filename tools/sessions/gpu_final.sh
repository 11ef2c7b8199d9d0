#!/bin/bash
# usage: tools/sessions/gpu_final.sh TAG -- round evidence: GPU tests, smoke, full bench (encoder blocks + CPU
# baseline), rocprofv3 kernel-trace stats (two-stream and single-stream), FETCH_SIZE / WRITE_SIZE passes.
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-run}
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
export UNET_OVERLAP=0
run prof1s 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_1s -- $B
unset UNET_OVERLAP
run pmcF 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $B
run pmcW 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $B
