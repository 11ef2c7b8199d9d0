# ConvTranspose data gradient + BN partials: 64-row tiles on under-filled grids (lab UNET_CONVT_BM64:
# 0 off, 1 64 x 64 tiles (default), 2 64 x 128) -- parity tests, then a same-box batch-8 A/B
set -e
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_ops_gpu.py -m gpu -k "convt or bn" > gpurun_out/cb_tests.log 2>&1
timeout -k 10 400 $T tests/test_model_gpu.py -m gpu > gpurun_out/cb_model.log 2>&1
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
C="python bench.py --num-classes 21 --batch 8 --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  for k in 0 1 2; do
    UNET_CONVT_BM64=$k timeout -k 10 300 $C > gpurun_out/cb_c4_${k}_$i.log 2>&1
  done
done
