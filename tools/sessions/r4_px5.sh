#!/bin/bash
# round 4: persistent forward with the gamma signs read once -- px tests, lab_px timing (bitwise vs
# the one-tile kernel), bench
source "$(dirname "$0")/gpu_session.sh"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run pxt 300 $T tests/test_ops_gpu.py -k "persistent or sepconv"
run px_check 240 python tools/lab_px.py 32 both
run c1 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run c1b 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
