#!/bin/bash
# Defaults changed (wave priority 3, deferred fused weight-gradient issue, unshuffle indexing):
# GPU tests, bench, kernel trace.
source "$(dirname "$0")/gpu_session.sh"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench1 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run bench2 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o x3 -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0
run convt 200 python tools/bench_convt.py
