#!/bin/bash
# round 4: the whole GPU suite + smoke + a bench line (no CPU baseline)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r4}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --no-cpu-baseline
