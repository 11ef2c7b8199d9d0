set -e
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "bwd_data_bnrelu or pointwise or train_step or convt" > gpurun_out/ab4_tests.log 2>&1
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B8="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0 --num-classes 21 --batch 8"
B16="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  UNET_BNBWD_BM64=0 timeout -k 10 300 $B8 > gpurun_out/ab4_c4b8_off_$i.log 2>&1
  UNET_BNBWD_BM64=1 timeout -k 10 300 $B8 > gpurun_out/ab4_c4b8_on_$i.log 2>&1
done
UNET_BNBWD_BM64=0 timeout -k 10 300 $B16 > gpurun_out/ab4_c1_off.log 2>&1
UNET_BNBWD_BM64=1 timeout -k 10 300 $B16 > gpurun_out/ab4_c1_on.log 2>&1
