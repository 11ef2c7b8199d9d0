#!/bin/bash
# usage: tools/sessions/ab_env.sh N "VAR=a" "VAR=b" -- alternate two environment settings, N benches each
source "$(dirname "$0")/gpu_session.sh"
N=$1; shift
for i in $(seq 1 "$N"); do
  for E in "$@"; do
    run bench 300 env "$E" python bench.py --steps 30 --warmup 5 --no-cpu-baseline --encoder-batch 0
    echo "AB $E $(grep -o '"value": [0-9.]*' gpurun_out/bench.log)"
  done
done
