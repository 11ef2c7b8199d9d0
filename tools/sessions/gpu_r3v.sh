#!/bin/bash
# enc2_block1 (64 -> 128) keeps no y (weight gradients recompute it): same-box step A/B
source "$(dirname "$0")/gpu_session.sh"
B="python bench.py --no-cpu-baseline --encoder-batch 0"
run a1 300 $B
run b1 300 $B --recompute-y64-128
run a2 300 $B
run b2 300 $B --recompute-y64-128
run a3 300 $B
run b3 300 $B --recompute-y64-128
