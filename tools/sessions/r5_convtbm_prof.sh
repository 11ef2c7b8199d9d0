# per-kernel durations of the ConvT data gradients (rows GEMM, A_UNSHUFFLE) at batch 8 / 16:
# UNET_CONVT_BM64 (64-row BN-partials tiles) x UNET_UNSHUFFLE_BK32 (32-deep k stages)
set -e
export UNET_HIP_LIB=$PWD/tools/labso/libunet_hip_lab.so
R=$PWD
cd /tmp && export TMPDIR=/tmp
C8="--num-classes 21 --batch 8"
for cfg in "1 0 8" "1 1 8" "0 1 8" "0 0 8" "1 0 16" "1 1 16"; do
  set -- $cfg
  A=""; [ "$3" = 8 ] && A="$C8"
  UNET_CONVT_BM64=$1 UNET_UNSHUFFLE_BK32=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cbq_$1$2_$3 -o run -- python3 $R/bench.py $A --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0 > $R/gpurun_out/cbq_$1$2_$3.log 2>&1
done
