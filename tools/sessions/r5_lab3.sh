set -e
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "convt_bwd_data_bnstats or dropout or train_step" > gpurun_out/lab3_tests.log 2>&1
cd tools/lab
for st in 0 256 512 1024 66048; do
  UNET_ROWS_KO=$st LAB_KO=$st LAB_MODE=1 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab3_m1_st$st.log 2>&1
done
for st in 0 512; do
  UNET_ROWS_KO=$st LAB_KO=$st LAB_MODE=0 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab3_m0_st$st.log 2>&1
  UNET_ROWS_KO=$st LAB_KO=$st LAB_MODE=3 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab3_m3_st$st.log 2>&1
done
cd ../..
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/lab3_ab_base_$i.log 2>&1
  UNET_ROWS_KO=512 timeout -k 10 300 $B > gpurun_out/lab3_ab_st512_$i.log 2>&1
  UNET_WGRAD_LDSPAD=21504 UNET_DWF_LDSPAD=9216 timeout -k 10 300 $B > gpurun_out/lab3_ab_p2_$i.log 2>&1
  UNET_BNBWD_BK16=1 UNET_WGRAD_LDSPAD=21504 UNET_DWF_LDSPAD=9216 timeout -k 10 300 $B > gpurun_out/lab3_ab_p2bk16_$i.log 2>&1
  UNET_BNBWD_BK16=1 UNET_WGRAD_LDSPAD=48300 UNET_DWF_LDSPAD=36100 timeout -k 10 300 $B > gpurun_out/lab3_ab_p1bk16_$i.log 2>&1
done
