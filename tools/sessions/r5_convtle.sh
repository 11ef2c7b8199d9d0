# ConvT BN-partials data gradient on 64-row tiles also at the batch-16 bottleneck (lab UNET_CONVT_BM64_LE=512: 1024 blocks) vs <= 256 (default)
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  for k in 256 512; do
    UNET_CONVT_BM64_LE=$k timeout -k 10 300 $B > gpurun_out/le_c1_${k}_$i.log 2>&1
  done
done
