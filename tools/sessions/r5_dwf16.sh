# depthwise filter-gradient persistent blocks 1024 (default) vs 512 at batch 16 (configs[1]), configs[4] batch 32 and configs[3]
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
D="python bench.py --num-classes 21 --batch 32 --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
E="python bench.py --size 512 --batch 8 --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3 4; do
  for k in 1024 512; do
    UNET_DWF_BLOCKS=$k timeout -k 10 300 $B > gpurun_out/d16_${k}_$i.log 2>&1
  done
done
for i in 1 2; do
  for k in 1024 512; do
    UNET_DWF_BLOCKS=$k timeout -k 10 300 $D > gpurun_out/d32_${k}_$i.log 2>&1
    UNET_DWF_BLOCKS=$k timeout -k 10 300 $E > gpurun_out/d512_${k}_$i.log 2>&1
  done
done
