#!/bin/bash
# usage: tools/sessions/r6_v.sh TAG -- validate HEAD: GPU tests, smoke, a short bench line, kernel-trace stats
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r6v}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --encoder-batch 0
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0 --no-roofline
