# deferred side-stream weight gradient issued after the next block's data-gradient launch (UNET_SW_LATE=1) vs before it
set -e
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  for k in 0 1; do
    UNET_SW_LATE=$k timeout -k 10 300 $B > gpurun_out/sl_c1_${k}_$i.log 2>&1
    UNET_SW_LATE=$k timeout -k 10 300 $C > gpurun_out/sl_c4_${k}_$i.log 2>&1
  done
done
