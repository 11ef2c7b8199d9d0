#!/bin/bash
# Rehearsal of the multi-rank bench path on one GPU (both ranks on device 0, gloo collectives).
source "$(dirname "$0")/gpu_session.sh"
UNET_DP_ONE_DEVICE=1 run dp2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0
# the driver's command shape: bench.py --gpus 2 without a launcher spawns the ranks itself
UNET_DP_ONE_DEVICE=1 run dp2spawn 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --encoder-batch 0
