set -e
cd tools/lab
for m in 1 0 2 3; do LAB_MODE=$m timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab1_mode$m.log 2>&1; done
UNET_ROWS_KO=7 LAB_KO=7 LAB_MODE=1 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab1_mode1_ko7.log 2>&1
LAB_WGRAD=1 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab1_wgrad.log 2>&1
cd ../..
UNET_PARITY_LOG=gpurun_out/r5a_parity.jsonl timeout -k 10 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -q --timeout 300 --timeout-method thread -k "training_geometry or relu_decisions" > gpurun_out/r5a_parity.log 2>&1
