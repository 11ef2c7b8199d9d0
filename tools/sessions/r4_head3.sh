#!/bin/bash
# round 4: fused head backward with batched loads, LDS-staged dice finalize -- tests + benches + trace
source "$(dirname "$0")/gpu_session.sh"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run ops 300 $T tests/test_ops_gpu.py -k "head or dice or meaniou"
run model 500 $T tests/test_model_gpu.py tests/test_parity_sizes_gpu.py
run c4 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --num-classes 21 --batch 8
run c1 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run c4tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4 -o c4 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8
run c1tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1 -o c1 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0
