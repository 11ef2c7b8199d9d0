#!/bin/bash
# usage: tools/sessions/gpu_full.sh TAG [gemm]  -- tests, bench, rocprof kernel stats (+ optional GEMM microbench)
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-run}
run ops 600 python -m pytest tests/test_ops_gpu.py -q -x
run model 900 python -m pytest tests/test_model_gpu.py -q -x
if [ "$2" == "gemm" ]; then run gemm 600 python tools/bench_gemm.py; fi
run bench 600 python bench.py --steps 20 --warmup 5
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $TAG -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
