#!/bin/bash
# Fused weight gradient on fewer CUs (its 111 KB of LDS per CU leaves co-running main-stream
# blocks one slot per CU): step A/B of the block count, plus a trace at 128 blocks.
source "$(dirname "$0")/gpu_session.sh"
run t_sw 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "sepconv_bwd_filter" --timeout 120 --timeout-method thread
for i in 1 2; do
  for V in base 128 192; do
    case $V in base) E="UNET_X=0" ;; *) E="UNET_SW_BLOCKS=$V" ;; esac
    run ab_${V}_$i 300 env $E python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB $V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab5.txt
  done
done
UNET_SW_BLOCKS=128 run prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o x5 -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0
