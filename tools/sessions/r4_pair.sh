#!/bin/bash
# round 4: weight-gradient slab pairs (pointwise + depthwise of the fused / filter-only backward, head kernel +
# bias) reduced in ONE launch (B, product build 79d6024d) vs two-three launches (A = c2b2c8b2), alternated; GPU tests on B
source "$(dirname "$0")/gpu_session.sh"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
B1="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
B4="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8"
for i in 1 2 3; do
  run b4A$i 200 env UNET_HIP_LIB=tools/lab/libunet_hip_A.so $B4
  run b4B$i 200 $B4
  run b1A$i 200 env UNET_HIP_LIB=tools/lab/libunet_hip_A.so $B1
  run b1B$i 200 $B1
done
grep -h '"value"' gpurun_out/b*.log | sed 's/.*"value": \([0-9.]*\).*/\1/' > /dev/null
for f in gpurun_out/b4A* gpurun_out/b4B* gpurun_out/b1A* gpurun_out/b1B*; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
