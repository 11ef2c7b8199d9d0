#!/bin/bash
# fused split-precision forward on every level (--fuse always) vs >= 64x64 only: same-box A/B
source "$(dirname "$0")/gpu_session.sh"
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run a1 300 $B
run b1 300 $B --fuse always
run a2 300 $B
run b2 300 $B --fuse always
run tests 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "fuse or always"
