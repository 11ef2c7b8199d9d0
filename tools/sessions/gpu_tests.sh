#!/bin/bash
# the round-end GPU checks: all GPU tests, smoke, default bench
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-final}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
