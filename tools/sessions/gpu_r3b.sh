#!/bin/bash
# PMC stall breakdown of the rows / wgrad GEMMs (fp32 vs bf16x6), CPU-baseline thread sweep, loader rates
source "$(dirname "$0")/gpu_session.sh"
LAB=tools/lab/libunet_hip_lab.so
export ITERS=3
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS"
for T in f32 x6; do
  if [ $T == x6 ]; then export UNET_HIP_LIB=$LAB UNET_X6=1; fi
  run pmc1_$T 300 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc -o rows1_$T -- python tools/bench_rows.py $T
  run pmc2_$T 300 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc -o rows2_$T -- python tools/bench_rows.py $T
done
unset UNET_HIP_LIB UNET_X6 ITERS
run cpusweep 600 python tools/cpu_sweep.py gpurun_out/cpu_sweep.jsonl 16 64 128
run loader 400 python tools/bench_loader.py gpurun_out/loader.jsonl 4 8 16
