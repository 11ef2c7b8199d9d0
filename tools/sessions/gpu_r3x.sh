#!/bin/bash
# rows-GEMM tile re-sweep after the XCD-grouped N-tiles (lab build: UNET_ROWS_BN / UNET_ROWS_BK override)
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/lab/libunet_hip_lab2.so
run def 300 env UNET_HIP_LIB=$LAB python tools/bench_rows.py def
run bn256 300 env UNET_HIP_LIB=$LAB UNET_ROWS_BN=256 UNET_ROWS_BK=16 python tools/bench_rows.py bn256
run bn128k16 300 env UNET_HIP_LIB=$LAB UNET_ROWS_BN=128 UNET_ROWS_BK=16 python tools/bench_rows.py bn128k16
run bn128k32 300 env UNET_HIP_LIB=$LAB UNET_ROWS_BN=128 UNET_ROWS_BK=32 python tools/bench_rows.py bn128k32
