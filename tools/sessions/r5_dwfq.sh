# depthwise filter-gradient blocks: 512 where a launch has <= UNET_DWF_SMALL_ITEMS tile-chunk items (0 = always 1024, the old default)
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 40 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
D="python bench.py --num-classes 21 --batch 32 --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
E="python bench.py --size 512 --batch 8 --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  for k in 0 4096 2048; do
    UNET_DWF_SMALL_ITEMS=$k timeout -k 10 300 $C > gpurun_out/dq_c4_${k}_$i.log 2>&1
    UNET_DWF_SMALL_ITEMS=$k timeout -k 10 300 $B > gpurun_out/dq_c1_${k}_$i.log 2>&1
  done
done
for i in 1 2; do
  for k in 0 4096 2048; do
    UNET_DWF_SMALL_ITEMS=$k timeout -k 10 300 $D > gpurun_out/dq_b32_${k}_$i.log 2>&1
    UNET_DWF_SMALL_ITEMS=$k timeout -k 10 300 $E > gpurun_out/dq_c3_${k}_$i.log 2>&1
  done
done
