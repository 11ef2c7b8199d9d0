# rows GEMM narrow-tile threshold (lab UNET_ROWS_NARROW_LT): < 256 blocks (default) vs <= 256 vs < 512
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $C > gpurun_out/nw_c4_256_$i.log 2>&1
  UNET_ROWS_NARROW_LT=257 timeout -k 10 300 $C > gpurun_out/nw_c4_257_$i.log 2>&1
  UNET_ROWS_NARROW_LT=512 timeout -k 10 300 $C > gpurun_out/nw_c4_512_$i.log 2>&1
  timeout -k 10 300 $B > gpurun_out/nw_c1_256_$i.log 2>&1
  UNET_ROWS_NARROW_LT=257 timeout -k 10 300 $B > gpurun_out/nw_c1_257_$i.log 2>&1
  UNET_ROWS_NARROW_LT=512 timeout -k 10 300 $B > gpurun_out/nw_c1_512_$i.log 2>&1
done
