#!/bin/bash
# usage: tools/sessions/gpu_abp.sh TAG "ENV=1" "ENV=0" -- tests, then per env setting a bench and a kernel-trace profile
source "$(dirname "$0")/gpu_session.sh"
TAG=$1; shift
run ops 600 python -m pytest tests/test_ops_gpu.py -q -x
run model 900 python -m pytest tests/test_model_gpu.py -q -x
i=0
for E in "$@"; do
  i=$((i+1))
  run bench_$i 600 env $E python bench.py --steps 20 --warmup 5 --no-cpu-baseline --encoder-batch 0
  grep -o '"value": [0-9.]*' gpurun_out/bench_$i.log | head -1
done
i=0
for E in "$@"; do
  i=$((i+1))
  export ${E%%=*}=${E#*=}
  run prof_$i 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_$i -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
done
