#!/bin/bash
# usage: tools/sessions/r6_y.sh -- round 6: split-precision rows GEMMs in the train step: x6 parity tests, the
# whole GPU suite, and the configs[1] step with / without them (alternated, same box)
source "$(dirname "$0")/gpu_session.sh"
export UNET_PARITY_LOG=gpurun_out/parity_r6y.jsonl
run x6tests 300 python -u -m pytest tests/test_x6_gpu.py -x -q --timeout 120 --timeout-method thread
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  run ab_x6_$i 300 $B
  run ab_f32_$i 300 $B --no-x6-gemm
done
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
