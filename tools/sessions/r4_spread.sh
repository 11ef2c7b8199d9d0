#!/bin/bash
# round 4: run-to-run spread of the end library on one box (configs[4] b8 and configs[1], 3 runs each)
source "$(dirname "$0")/gpu_session.sh"
B1="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
B4="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8"
for i in 1 2 3; do
  run s4_$i 200 $B4
  run s1_$i 200 $B1
done
for f in gpurun_out/s4_* gpurun_out/s1_*; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
