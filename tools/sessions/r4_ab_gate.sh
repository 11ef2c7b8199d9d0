#!/bin/bash
# round 4: A/B of the side-GEMM gate (UNET_GATE_GEMM=1 vs 0), alternating, same box
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2 3; do
  for G in 1 0; do
    run ab_${G}_$i 300 env UNET_GATE_GEMM=$G python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB gate=$G $(grep -o '"value": [0-9.]*' gpurun_out/ab_${G}_$i.log)" | tee -a gpurun_out/ab_gate.txt
  done
done
run ab_cfg4_1 300 env UNET_GATE_GEMM=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
run ab_cfg4_0 300 env UNET_GATE_GEMM=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
echo "cfg4 gate=1 $(grep -o '"value": [0-9.]*' gpurun_out/ab_cfg4_1.log) gate=0 $(grep -o '"value": [0-9.]*' gpurun_out/ab_cfg4_0.log)" | tee -a gpurun_out/ab_gate.txt
