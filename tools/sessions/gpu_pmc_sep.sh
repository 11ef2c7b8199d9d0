#!/bin/bash
# PMC passes (one counter group per run; kernel-trace only) on fused sepconv shapes
source "$(dirname "$0")/gpu_session.sh"
for S in "1 128 128 128 128" "1 32 32 512 512"; do
  T=$(echo $S | tr ' ' '_')
  run pmc1_$T 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc -o s1_$T -- python tools/sep_one.py $S 10 $1
  run pmc2_$T 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc -o s2_$T -- python tools/sep_one.py $S 10 $1
  run pmc3_$T 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc -o s3_$T -- python tools/sep_one.py $S 10 $1
  run pmc4_$T 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o s4_$T -- python tools/sep_one.py $S 10 $1
  run pmc5_$T 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o s5_$T -- python tools/sep_one.py $S 10 $1
done
