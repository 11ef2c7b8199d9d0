#!/bin/bash
# round 4: fused multi-class head backward (packed FMAs), MFMA head forward, LDS-staged dice sums,
# 64-wide N tiles for under-filled rows GEMMs -- op / model / parity tests, then configs[4] b8 and
# configs[1] benches with the narrow-tile rule on and off (lab library knob)
source "$(dirname "$0")/gpu_session.sh"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run ops 400 $T tests/test_ops_gpu.py
run model 500 $T tests/test_model_gpu.py tests/test_parity_sizes_gpu.py
B4="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --num-classes 21 --batch 8"
B1="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline"
run c4 200 $B4
run c1 200 $B1
export UNET_HIP_LIB=tools/lab/libunet_hip_lab.so
run c4_n0 200 env UNET_ROWS_NARROW=0 $B4
run c4_n1 200 env UNET_ROWS_NARROW=1 $B4
run c1_n0 200 env UNET_ROWS_NARROW=0 $B1
run c1_n1 200 env UNET_ROWS_NARROW=1 $B1
unset UNET_HIP_LIB
run c4tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4 -o c4 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
