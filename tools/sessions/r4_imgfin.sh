#!/bin/bash
# round 4: image block final weight-gradient reduction with all 32 row loads in flight (B, product build)
# vs the one-row-at-a-time final (A = a106ce36), alternated
source "$(dirname "$0")/gpu_session.sh"
run timg 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "image_block or pointwise_bwd_data_bnrelu_wgrad"
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
