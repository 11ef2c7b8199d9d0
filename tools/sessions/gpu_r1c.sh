#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run model21 600 python -m pytest tests/test_model_gpu.py -q -x -k "21" -s
run gemm 600 python tools/bench_gemm.py
