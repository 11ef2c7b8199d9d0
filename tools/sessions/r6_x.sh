#!/bin/bash
# usage: tools/sessions/r6_x.sh -- round 6: split-precision (bf16x6) rows GEMMs with pre-split weight planes,
# BK 32 single-buffer stages (gemm.hip X6) vs the fp32-MFMA route, per train-step shape; x6 parity tests
source "$(dirname "$0")/gpu_session.sh"
run x6tests 300 python -u -m pytest tests/test_x6_gpu.py -x -q --timeout 120 --timeout-method thread
run x6bench 300 python tools/bench_dgrad_x6.py x6
run x6bench_drop 300 env DROP=0.2 python tools/bench_dgrad_x6.py x6drop
