#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run gtests 900 python -m pytest tests -q -m gpu
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r1d -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
