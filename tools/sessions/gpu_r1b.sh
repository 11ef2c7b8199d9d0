#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run ops 600 python -m pytest tests/test_ops_gpu.py -q -x
run model 900 python -m pytest tests/test_model_gpu.py -q -x
run bench 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r1b -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
