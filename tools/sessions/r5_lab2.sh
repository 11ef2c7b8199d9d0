set -e
cd tools/lab
timeout -k 10 120 ./mfma_ceiling > ../../gpurun_out/lab2_ceiling.log 2>&1
cd ../..
export TMPDIR=/tmp
for s in 15 9; do
  LAB_SHAPE=$s timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc2 -o s$s-p1 -- ./tools/lab/gemm_lab > gpurun_out/lab2_pmc_s$s.log 2>&1
done
cd tools/lab
LAB_MODE=1 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab2_mode1_nodrop.log 2>&1
UNET_ROWS_KO=7 LAB_KO=7 LAB_MODE=1 timeout -k 10 240 ./gemm_lab > ../../gpurun_out/lab2_mode1_nodrop_ko7.log 2>&1
cd ../..
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/lab2_ab_base_$i.log 2>&1
  UNET_BNBWD_BK16=1 timeout -k 10 300 $B > gpurun_out/lab2_ab_bk16_$i.log 2>&1
done
