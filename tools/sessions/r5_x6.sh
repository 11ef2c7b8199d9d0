# split-precision (bf16x6) rows / weight-gradient GEMMs in the step (lab build, UNET_X6=1) vs fp32 MFMA
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B16="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B16 > gpurun_out/x6_base_$i.log 2>&1
  UNET_X6=1 timeout -k 10 300 $B16 > gpurun_out/x6_on_$i.log 2>&1
done
