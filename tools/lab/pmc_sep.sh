#!/bin/bash
# PMC passes over the sepconv lab (one shape): old vs register-A kernel
cd "$(dirname "$0")"
export TMPDIR=/tmp
O=../../gpurun_out/pmc_sep
mkdir -p $O
run() { timeout -s KILL 60 rocprofv3 --pmc $2 --output-format csv -d $O -o $1 -- ./sep_rk_lab 3 one > $O/$1.log 2>&1; echo "$1 rc=$?"; }
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
run p2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_INSTS_SALU"
run p3 "GRBM_GUI_ACTIVE GRBM_COUNT"
