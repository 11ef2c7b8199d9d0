#!/bin/bash
# usage: tools/sessions/r6_b.sh TAG -- round 6: GPU tests (persistent rows GEMM, the batch-32 fixture),
# per-shape rows-GEMM times with the persistent tile stream off / on (lab library), a same-box step
# A/B (UNET_ROWS_PERS 0 / 1, alternated), and the product bench line
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r6b}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
LAB=tools/labbin/libunet_hip_lab.so
run rows_p0 300 env UNET_HIP_LIB=$LAB UNET_ROWS_PERS=0 python tools/bench_rows.py pers0
run rows_p1 300 env UNET_HIP_LIB=$LAB UNET_ROWS_PERS=1 python tools/bench_rows.py pers1
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  run ab_p0_$i 300 env UNET_HIP_LIB=$LAB UNET_ROWS_PERS=0 $B
  run ab_p1_$i 300 env UNET_HIP_LIB=$LAB UNET_ROWS_PERS=1 $B
done
run bench 600 python bench.py --no-cpu-baseline
