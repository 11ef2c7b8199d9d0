#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run smoke 420 python -c "import __graft_entry__ as g; g.smoke()"
run ops 600 python -m pytest tests/test_ops_gpu.py -q -x
run model 900 python -m pytest tests/test_model_gpu.py -q
run bench 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r1a -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
