#!/bin/bash
# usage: tools/sessions/r6_v2.sh -- round 6: x6 tests (64-column tiles for <= 64 output columns), per-shape rows
# A/B, and the encoder-block table (batch 32) with the y stores left in flight (current) vs waited (base library)
source "$(dirname "$0")/gpu_session.sh"
run x6tests 300 python -u -m pytest tests/test_x6_gpu.py -x -q --timeout 120 --timeout-method thread
run x6bench 300 python tools/bench_dgrad_x6.py x6n64
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 32"
run enc_yw1 300 $B
run enc_yw0 300 env UNET_HIP_LIB=$PWD/tools/labbin/libunet_hip_base.so $B
run enc_yw1b 300 $B
run enc_yw0b 300 env UNET_HIP_LIB=$PWD/tools/labbin/libunet_hip_base.so $B
