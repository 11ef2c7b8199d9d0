#!/bin/bash
# round 4: dice finalize with 8-lane term groups; head backward dice coefficients from LDS
source "$(dirname "$0")/gpu_session.sh"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run ops 300 $T tests/test_ops_gpu.py -k "head or dice or meaniou"
run model 500 $T tests/test_model_gpu.py tests/test_parity_sizes_gpu.py
run lab 200 env UNET_HIP_LIB=tools/lab/libunet_hip_lab.so python tools/lab_head.py 0
B4="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --num-classes 21 --batch 8 --encoder-batch 0"
run c4a 200 $B4
run c4b 200 $B4
run c1 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
run c4tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4 -o c4 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
