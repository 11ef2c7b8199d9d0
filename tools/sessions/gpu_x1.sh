#!/bin/bash
# Round-2 experiment session: step traces (base / raised main-stream wave priority / deferred fused
# weight-gradient issue), bench A/B of the same plus a 256-block weight-gradient grid, and a
# Conv2DTranspose tile sweep.
source "$(dirname "$0")/gpu_session.sh"
L=unet-image-segmentation_amd/unet_amd
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0"
run prof_base 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o base -- $B
UNET_HIP_LIB=$L/libunet_hip_prio.so run prof_prio 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o prio -- $B
UNET_SW_DEFER=1 run prof_defer 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o defer -- $B
for i in 1 2; do
  for V in base defer prio wg256; do
    case $V in
      base) E="UNET_X=0" ;; defer) E="UNET_SW_DEFER=1" ;; prio) E="UNET_HIP_LIB=$L/libunet_hip_prio.so" ;;
      wg256) E="UNET_WGRAD_BLOCKS=256" ;;
    esac
    run ab_${V}_$i 300 env $E python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
    echo "AB $V $(grep -o '"value": [0-9.]*' gpurun_out/ab_${V}_$i.log)" | tee -a gpurun_out/ab.txt
  done
done
for C in default 128,16 128,32 256,16 64,32; do
  if [ $C = default ]; then run convt_$C 200 python tools/bench_convt.py
  else UNET_ROWS_CFG=$C run convt_$C 200 python tools/bench_convt.py; fi
done
