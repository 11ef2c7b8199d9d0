# batch-aware fusion of the 32x32 level: model tests, then configs[1] / configs[4] b32 vs HEAD and the encoder table
set -e
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_model_gpu.py tests/test_parity_sizes_gpu.py -m gpu > gpurun_out/f32_tests.log 2>&1
B="--steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
C="--num-classes 21 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 python tools/abhead/bench.py $B > gpurun_out/f32_head_$i.log 2>&1
  timeout -k 10 300 python bench.py $B > gpurun_out/f32_new_$i.log 2>&1
  timeout -k 10 300 python tools/abhead/bench.py $C > gpurun_out/f32_c4head_$i.log 2>&1
  timeout -k 10 300 python bench.py $C > gpurun_out/f32_c4new_$i.log 2>&1
done
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/f32_table.log 2>&1
