#!/bin/bash
# usage: tools/sessions/r6_h.sh -- round 6: with the LDS-DMA split-precision forward (r6g: 32^2 launch
# 54.8 -> 47.3 us), does the fused forward now pay on the 32 x 32 level at batch 16 (configs[1]) and
# batch 8 (configs[4] per GPU)?  UNET_FUSE_MIN_TOTAL = 16384 / 8192 vs the default 32768, alternated (the round-6
# library read that variable at import; later ones take bench.py --fuse-min-total instead).
source "$(dirname "$0")/gpu_session.sh"
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
B4="$B --num-classes 21 --batch 8"
for i in 1 2 3; do
  run c1_def_$i 300 $B
  run c1_f16k_$i 300 env UNET_FUSE_MIN_TOTAL=16384 $B
done
for i in 1 2; do
  run c4_def_$i 300 $B4
  run c4_f8k_$i 300 env UNET_FUSE_MIN_TOTAL=8192 $B4
done
export UNET_FUSE_MIN_TOTAL=16384
run tests 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread -k "train256"
