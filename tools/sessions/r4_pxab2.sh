#!/bin/bash
# round 4: the persistent forward restricted to its in-step winners (AUTO) vs off (lab UNET_PX=0),
# configs[1] alternated on one box, a kernel trace of each, and the px tests
source "$(dirname "$0")/gpu_session.sh"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run pxt 300 $T tests/test_ops_gpu.py -k "persistent or sepconv"
B1="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
for r in 1 2 3; do
  run auto_$r 200 env UNET_PX=1 $B1
  run off_$r 200 env UNET_PX=0 $B1
done
unset UNET_HIP_LIB
run tr 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pxab -o auto -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0
