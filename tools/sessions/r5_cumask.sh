# side stream on a CU-masked queue (lab build): none / full mask (queue cost alone) / every 16th,
# 8th, 4th CU reserved for the main stream's launches
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B16="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B16 > gpurun_out/cm_base_$i.log 2>&1
  UNET_SIDE_CUMASK=0 timeout -k 10 300 $B16 > gpurun_out/cm_full_$i.log 2>&1
  UNET_SIDE_CUMASK=16 timeout -k 10 300 $B16 > gpurun_out/cm_16_$i.log 2>&1
  UNET_SIDE_CUMASK=8 timeout -k 10 300 $B16 > gpurun_out/cm_8_$i.log 2>&1
  UNET_SIDE_CUMASK=4 timeout -k 10 300 $B16 > gpurun_out/cm_4_$i.log 2>&1
done
