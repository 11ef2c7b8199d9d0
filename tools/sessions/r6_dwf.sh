#!/bin/bash
# usage: tools/sessions/r6_dwf.sh -- round 6: the BN+ReLU-view blocks' depthwise filter gradient inside their
# depthwise data-gradient pass (unet_dwconv3x3_bwd_data_bnstats_dwf) vs its own side-stream pass: tests, the
# configs[1] step and configs[4] per GPU, alternated on one box
source "$(dirname "$0")/gpu_session.sh"
run dwftests 300 python -u -m pytest tests/test_dwf_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  run ab_dwf1_$i 300 $B
  run ab_dwf0_$i 300 $B --no-dw-fused-filter
done
run ab_c4_dwf1 300 $B --num-classes 21 --batch 8
run ab_c4_dwf0 300 $B --num-classes 21 --batch 8 --no-dw-fused-filter
