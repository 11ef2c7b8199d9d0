# In-launch BatchNorm finish: tests, then step A/B (product lib on/off; lab lib per producer class)
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_fin_gpu.py > gpurun_out/fin2_tests.log 2>&1
B16="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B16 > gpurun_out/fin2_on_$i.log 2>&1
  timeout -k 10 300 $B16 --no-fin-in-launch > gpurun_out/fin2_off_$i.log 2>&1
done
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
UNET_FIN_GEMM=0 timeout -k 10 300 $B16 > gpurun_out/fin2_nogemm.log 2>&1
UNET_FIN_RK=0 timeout -k 10 300 $B16 > gpurun_out/fin2_nork.log 2>&1
UNET_FIN_PX=0 timeout -k 10 300 $B16 > gpurun_out/fin2_nopx.log 2>&1
