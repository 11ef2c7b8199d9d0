#!/bin/bash
# round-3 session: GPU tests, bench (+ encoder table), PMC stall breakdown of the GEMMs, CPU sweep, loader
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3c}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 400 python bench.py --no-cpu-baseline
LAB=tools/lab/libunet_hip_lab.so
export ITERS=3
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS"
run pmc1_f32 300 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc -o rows1_f32 -- python tools/bench_rows.py f32
run pmc2_f32 300 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc -o rows2_f32 -- python tools/bench_rows.py f32
unset ITERS
run cpusweep 600 python tools/cpu_sweep.py gpurun_out/cpu_sweep.jsonl 16 64 128
run loader 400 python tools/bench_loader.py gpurun_out/loader.jsonl 4 8 16
