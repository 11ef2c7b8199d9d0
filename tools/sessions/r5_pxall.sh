# persistent forward on every supported shape (lab UNET_PX_ALL=1) at configs[4] batch 8 and configs[1]
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $C > gpurun_out/pa_c4_base_$i.log 2>&1
  UNET_PX_ALL=1 timeout -k 10 300 $C > gpurun_out/pa_c4_all_$i.log 2>&1
done
timeout -k 10 300 $B > gpurun_out/pa_c1_base.log 2>&1
UNET_PX_ALL=1 timeout -k 10 300 $B > gpurun_out/pa_c1_all.log 2>&1
