#!/bin/bash
# Fused 64-output block backward: knock-out decomposition and PMC (SQ counters) of the product kernel
source "$(dirname "$0")/gpu_session.sh"
for k in 0 1 16 17 2 4 8 32; do run swko$k 60 tools/lab/sw_fused_ko$k; done
cd tools/lab
P=../../gpurun_out/pmc_sw; mkdir -p $P
run pmcsw1 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_WAIT_INST_ANY --output-format csv -d $P -o p1 -- ./sw_fused_ko0
run pmcsw2 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $P -o p2 -- ./sw_fused_ko0
run pmcsw3 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P -o p3 -- ./sw_fused_ko0
run pmcsw4 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P -o p4 -- ./sw_fused_ko0
