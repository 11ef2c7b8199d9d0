# side-stream grid re-sweep on the round-5 tree (lab): default vs fewer / longer weight-gradient blocks
# (UNET_WGRAD_BLOCKS=512 UNET_WGRAD_MINROWS=1024) vs depthwise filter-gradient blocks 512 / 2048 (UNET_DWF_BLOCKS)
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/sg_c1_def_$i.log 2>&1
  UNET_WGRAD_BLOCKS=512 UNET_WGRAD_MINROWS=1024 timeout -k 10 300 $B > gpurun_out/sg_c1_wg512_$i.log 2>&1
  UNET_DWF_BLOCKS=512 timeout -k 10 300 $B > gpurun_out/sg_c1_dwf512_$i.log 2>&1
  UNET_DWF_BLOCKS=2048 timeout -k 10 300 $B > gpurun_out/sg_c1_dwf2048_$i.log 2>&1
  timeout -k 10 300 $C > gpurun_out/sg_c4_def_$i.log 2>&1
  UNET_WGRAD_BLOCKS=512 UNET_WGRAD_MINROWS=1024 timeout -k 10 300 $C > gpurun_out/sg_c4_wg512_$i.log 2>&1
  UNET_DWF_BLOCKS=512 timeout -k 10 300 $C > gpurun_out/sg_c4_dwf512_$i.log 2>&1
  UNET_DWF_BLOCKS=2048 timeout -k 10 300 $C > gpurun_out/sg_c4_dwf2048_$i.log 2>&1
done
