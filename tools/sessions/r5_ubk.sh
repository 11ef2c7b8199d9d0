# ConvT data gradient BK 32 only on narrow (64-column) grids (lab UNET_UNSHUFFLE_BK32=2: the bottleneck at batch 16) vs 16 (default)
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 40 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  for k in 0 2; do
    UNET_UNSHUFFLE_BK32=$k timeout -k 10 300 $B > gpurun_out/ub_c1_${k}_$i.log 2>&1
    UNET_UNSHUFFLE_BK32=$k timeout -k 10 300 $C > gpurun_out/ub_c4_${k}_$i.log 2>&1
  done
done
