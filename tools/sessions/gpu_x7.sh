#!/bin/bash
# MeanIoU update on the side stream, one-wave-per-term dice finalize, options removed: GPU tests,
# bench x2, kernel trace.
source "$(dirname "$0")/gpu_session.sh"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench1 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run bench2 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o x7 -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0
