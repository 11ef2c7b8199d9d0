#!/bin/bash
# usage: tools/sessions/gpu_final3.sh TAG -- round-3 evidence: GPU tests, smoke, full bench (encoder table + CPU
# baseline), rocprofv3 kernel-trace stats (two-stream and single-stream), FETCH_SIZE / WRITE_SIZE
# passes of the bench, and a PMC group on enc2_block1's forward at batch 32
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3z}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
export UNET_OVERLAP=0
run prof1s 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_1s -- $B
unset UNET_OVERLAP
run pmcF 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $B
run pmcW 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $B
export N=32
S="python tools/sep_one.py 1 128 128 64 128 10 x3"
run sepF 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e2b1_fetch -- $S
run sepW 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e2b1_write -- $S
run sepS 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc -o ${TAG}_e2b1_sq -- $S
