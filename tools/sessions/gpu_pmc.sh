#!/bin/bash
# PMC passes (one counter group per run; kernel-trace only) on one GEMM shape
source "$(dirname "$0")/gpu_session.sh"
S="fwd 262144 512 256"
run pmc1 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc -o p1 -- python tools/gemm_one.py $S
run pmc2 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc -o p2 -- python tools/gemm_one.py $S
run pmc3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o p3 -- python tools/gemm_one.py $S
run pmc4 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o p4 -- python tools/gemm_one.py $S
