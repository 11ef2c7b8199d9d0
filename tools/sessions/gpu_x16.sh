#!/bin/bash
# Confirm the package default (HIP_FORCE_DEV_KERNARG set by unet_amd / bench.py) against an
# explicit 0; model tests under the default.
source "$(dirname "$0")/gpu_session.sh"
for i in 1 2; do
  run ab_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
  echo "AB default $(grep -o '"value": [0-9.]*' gpurun_out/ab_def_$i.log)" | tee -a gpurun_out/ab16.txt
  run ab_0_$i 300 env HIP_FORCE_DEV_KERNARG=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
  echo "AB explicit0 $(grep -o '"value": [0-9.]*' gpurun_out/ab_0_$i.log)" | tee -a gpurun_out/ab16.txt
done
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
