#!/bin/bash
# round 3: register-A fused forward without scratch spills -- A (HEAD: 128-column split-precision
# tile at 3 waves/SIMD, 66-114 VGPRs spilled), B (that tile at 2 waves: no spills), C (B, 128-column
# tiles also for >= 256 outputs), D (B, 64-column tile at 2 waves too); step A/B alternating
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2; do
  for v in A B C D; do
    UNET_HIP_LIB=$PWD/tools/lab/librk_$v.so run bench_${v}$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    grep -o '"value": [0-9.]*' gpurun_out/bench_${v}$i.log | head -1
  done
done
