# bn_finalize with its loads batched (one round trip per phase): parity suites, then same-box A/B vs HEAD
set -e
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_parity_sizes_gpu.py -m gpu > gpurun_out/fin7_tests.log 2>&1
B="--steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  timeout -k 10 300 python tools/abhead/bench.py $B > gpurun_out/fin7_head_$i.log 2>&1
  timeout -k 10 300 python bench.py $B > gpurun_out/fin7_new_$i.log 2>&1
done
