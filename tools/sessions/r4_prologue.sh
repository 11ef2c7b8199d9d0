#!/bin/bash
# round 4: the step prologue copies (image padding + padded image-block kernels) in one launch (B, default)
# vs three launches (A, UNET_PROLOGUE_BATCH=0); same library; GPU tests first
source "$(dirname "$0")/gpu_session.sh"
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
B1="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
B4="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8"
for i in 1 2 3; do
  run b4A$i 200 env UNET_PROLOGUE_BATCH=0 $B4
  run b4B$i 200 $B4
  run b1A$i 200 env UNET_PROLOGUE_BATCH=0 $B1
  run b1B$i 200 $B1
done
grep -h '"value"' gpurun_out/b*.log | sed 's/.*"value": \([0-9.]*\).*/\1/' > /dev/null
for f in gpurun_out/b4A* gpurun_out/b4B* gpurun_out/b1A* gpurun_out/b1B*; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
