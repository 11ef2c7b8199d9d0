# Upper bound of folding the BatchNorm statistics launches into their producers: the step with the
# 18 bn_finalize and/or 18 bn_bwd_stats launches skipped (lab build; numerics not meaningful).
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
B16="python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2; do
  timeout -k 10 300 $B16 > gpurun_out/ab6_base_$i.log 2>&1
  UNET_SKIP_BNFIN=1 timeout -k 10 300 $B16 > gpurun_out/ab6_nofin_$i.log 2>&1
  UNET_SKIP_BNBWD=1 timeout -k 10 300 $B16 > gpurun_out/ab6_nobwd_$i.log 2>&1
  UNET_SKIP_BNFIN=1 UNET_SKIP_BNBWD=1 timeout -k 10 300 $B16 > gpurun_out/ab6_none_$i.log 2>&1
done
