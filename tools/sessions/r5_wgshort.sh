# shorter side-stream weight-gradient blocks (lab UNET_WGRAD_MINROWS / UNET_WGRAD_BLOCKS): default 512 / 1024 vs 256 / 2048 vs 128 / 2048
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  for k in "512 1024" "256 2048" "128 2048"; do
    set -- $k
    UNET_WGRAD_MINROWS=$1 UNET_WGRAD_BLOCKS=$2 timeout -k 10 300 $B > gpurun_out/ws_c1_$1_$2_$i.log 2>&1
    UNET_WGRAD_MINROWS=$1 UNET_WGRAD_BLOCKS=$2 timeout -k 10 300 $C > gpurun_out/ws_c4_$1_$2_$i.log 2>&1
  done
done
