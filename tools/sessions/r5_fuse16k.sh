# configs[1] (batch 16) with the 32x32 level fused + split precision too (threshold 16384 pixels) vs 32768
set -e
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/f16_base_$i.log 2>&1
  UNET_FUSE_MIN_TOTAL=16384 timeout -k 10 300 $B > gpurun_out/f16_16k_$i.log 2>&1
  UNET_FUSE_MIN_TOTAL=8192 timeout -k 10 300 $B > gpurun_out/f16_8k_$i.log 2>&1
done
timeout -k 10 300 $C > gpurun_out/f16_c4_base.log 2>&1
UNET_FUSE_MIN_TOTAL=8192 timeout -k 10 300 $C > gpurun_out/f16_c4_8k.log 2>&1
