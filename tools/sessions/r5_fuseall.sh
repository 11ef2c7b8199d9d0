# fused forward on every level (incl. 32x32 / 16x16) vs AUTO: step and encoder table
set -e
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline"
timeout -k 10 400 $B > gpurun_out/fa_auto.log 2>&1
timeout -k 10 400 $B --fuse always > gpurun_out/fa_always.log 2>&1
