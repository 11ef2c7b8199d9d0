#!/bin/bash
# round 4: compute-only knock-outs + PMC of the persistent vs one-tile forward on enc2_block2 (batch 32)
source "$(dirname "$0")/gpu_session.sh"
run ko 400 tools/lab/x6_ko_lab 32
export N=32
S="python tools/sep_one.py 1 128 128 128 128 10 x3"
for SC in 3 0; do
  export SCHED=$SC
  run pmcA_$SC 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc -o px_A_$SC -- $S
  run pmcB_$SC 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc -o px_B_$SC -- $S
  run pmcF_$SC 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o px_F_$SC -- $S
  run pmcW_$SC 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o px_W_$SC -- $S
done
