# depthwise filter-gradient persistent blocks at batch 8 (configs[4]): 1024 (default) vs 512 vs 768, interleaved
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 40 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3 4; do
  for k in 1024 512 768; do
    UNET_DWF_BLOCKS=$k timeout -k 10 300 $C > gpurun_out/d8_${k}_$i.log 2>&1
  done
done
