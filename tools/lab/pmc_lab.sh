#!/bin/bash
# PMC passes over one lab shape: usage tools/lab/pmc_lab.sh SHAPE_INDEX TAG
source "$(dirname "$0")/../gpu_session.sh"
export LAB_SHAPE=$1
T=$2
run p1_$T 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc -o $T-p1 -- ./tools/lab/gemm_lab
run p2_$T 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc -o $T-p2 -- ./tools/lab/gemm_lab
