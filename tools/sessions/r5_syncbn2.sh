set -e
export UNET_DP_ONE_DEVICE=1 DP_CHECK_GLOBAL=5
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/dp_syncbn_check.py > gpurun_out/syncbn_sync.log 2>&1
