# SyncBN (SURVEY 8(e) option): op tests, the two-rank full-batch equality, and the per-replica
# (local BN) variant of the same comparison for contrast
set -e
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_ops_gpu.py -k "bn_sync or pointwise_and_bn" > gpurun_out/syncbn_tests.log 2>&1
timeout -k 10 900 $T tests/test_dp_gpu.py >> gpurun_out/syncbn_tests.log 2>&1
export UNET_DP_ONE_DEVICE=1 DP_CHECK_GLOBAL=5 DP_CHECK_LOCAL=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/dp_syncbn_check.py > gpurun_out/syncbn_local.log 2>&1
unset DP_CHECK_LOCAL
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/dp_syncbn_check.py > gpurun_out/syncbn_sync.log 2>&1
