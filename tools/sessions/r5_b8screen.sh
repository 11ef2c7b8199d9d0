# configs[4] batch 8 knob screen on the final tree (lab): default vs BN-backward GEMM BK 16, BK-32 K threshold 128 / 512, depthwise filter blocks 384
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 40 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  timeout -k 10 300 $C > gpurun_out/s8_def_$i.log 2>&1
  UNET_BNBWD_BK16=1 timeout -k 10 300 $C > gpurun_out/s8_bk16_$i.log 2>&1
  UNET_BK32_MIN_K=128 timeout -k 10 300 $C > gpurun_out/s8_k128_$i.log 2>&1
  UNET_BK32_MIN_K=512 timeout -k 10 300 $C > gpurun_out/s8_k512_$i.log 2>&1
  UNET_DWF_BLOCKS=384 timeout -k 10 300 $C > gpurun_out/s8_dwf384_$i.log 2>&1
done
