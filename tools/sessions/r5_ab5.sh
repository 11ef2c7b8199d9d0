set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B16="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B16 > gpurun_out/ab5_base_$i.log 2>&1
  UNET_DWF_BLOCKS=256 timeout -k 10 300 $B16 > gpurun_out/ab5_dwf256_$i.log 2>&1
  UNET_DWF_BLOCKS=512 timeout -k 10 300 $B16 > gpurun_out/ab5_dwf512_$i.log 2>&1
  UNET_WGRAD_MINROWS=256 UNET_WGRAD_BLOCKS=2048 timeout -k 10 300 $B16 > gpurun_out/ab5_wg256_$i.log 2>&1
done
