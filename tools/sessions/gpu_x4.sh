#!/bin/bash
# 128-output fused weight gradient (y recomputed at the 128 x 128 level) and enc1_block2's weight
# gradients on the main stream: op tests, then step A/B.
source "$(dirname "$0")/gpu_session.sh"
run t_sw 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "sepconv_bwd_filter" --timeout 120 --timeout-method thread
for i in 1 2; do
  for V in base y128 tail both; do
    case $V in
      base) E="UNET_X=0" ;; y128) E="UNET_RECOMPUTE_Y128=1" ;; tail) E="UNET_TAIL_MAIN=1" ;;
      both) E="UNET_RECOMPUTE_Y128=1 UNET_TAIL_MAIN=1" ;;
    esac
    run ab_${V}_$i 300 env $E python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB $V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab4.txt
  done
done
UNET_RECOMPUTE_Y128=1 UNET_TAIL_MAIN=1 run prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o x4 -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0
