# encoder table (batch 32) with the fused forward on every level vs AUTO, and configs[4] batch 32
set -e
B="python bench.py --steps 10 --warmup 5 --no-cpu-baseline"
timeout -k 10 400 $B > gpurun_out/fa2_auto.log 2>&1
timeout -k 10 400 $B --fuse always > gpurun_out/fa2_always.log 2>&1
C="python bench.py --num-classes 21 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
timeout -k 10 300 $C > gpurun_out/fa2_c4b32_auto.log 2>&1
timeout -k 10 300 $C --fuse always > gpurun_out/fa2_c4b32_always.log 2>&1
