#!/bin/bash
# usage: tools/sessions/r6_a.sh TAG -- round 6 first pass: GPU tests (the new dropout fixture), a short
# bench, and PMC groups on enc3_block1 / enc3_block2's fused forward at batch 32
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r6a}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not train256b32"
run bench 600 python bench.py --no-cpu-baseline
export N=32
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
S1="python tools/sep_one.py 1 64 64 128 256 10 x3"
run e3b1_sq 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b1_sq -- $S1
run e3b1_f 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b1_fetch -- $S1
export POOL=1
S2="python tools/sep_one.py 1 64 64 256 256 10 x3"
run e3b2_sq 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b2_sq -- $S2
run e3b2_f 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b2_fetch -- $S2
run e3b2_w 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b2_write -- $S2
run e3b2_kt 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b2_kt -- $S2
