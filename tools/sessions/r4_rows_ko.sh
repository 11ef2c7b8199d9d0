#!/bin/bash
# round 4: rows-GEMM knock-outs on the train step's shapes (lab library): 1 no C stores, 2 no dz
# side copy, 4 no k-loop operand loads
source "$(dirname "$0")/gpu_session.sh"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
for K in 0 1 2 3 4 7; do
  run rows_ko$K 300 env UNET_ROWS_KO=$K python tools/bench_rows.py ko$K
done
