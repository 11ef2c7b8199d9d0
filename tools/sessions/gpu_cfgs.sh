#!/bin/bash
# The other BASELINE configs at their per-GPU shape on one GPU (configs[3]: 512x512 batch 8;
# configs[4]: 21 classes batch 8, and its whole batch of 32), full train step, no CPU baseline.
source "$(dirname "$0")/gpu_session.sh"
run cfg3 300 python bench.py --size 512 --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run cfg4_b8 300 python bench.py --num-classes 21 --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run cfg4_b32 300 python bench.py --num-classes 21 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run cfg0 300 python bench.py --size 128 --batch 2 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
