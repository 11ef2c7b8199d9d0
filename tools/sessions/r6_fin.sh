#!/bin/bash
# usage: tools/sessions/r6_fin.sh TAG [A|B|C] -- (A: up to the step PMC passes; B: the PMC groups and other configs;
# C: the default bench line again once the PMC traffic summary of this library build is committed, so its
# roofline object carries the measured traffic -> profiles/r6fin_bench_pinned.log;
# S (commit 035656c, reverted after it: the route and its flag are gone): the fused 64-output block backward on the split-precision route -- its GPU tests, the training-
# geometry parity, then three alternated bench pairs against --no-x6-fused-bwd -> profiles/r6sx_*;
# G: inference through the captured HIP graph -- its GPU test, then eager vs graph latency -> profiles/r6g_*)
# round-6 evidence at HEAD: GPU tests, smoke, the full bench line
# (encoder table + CPU baseline), rocprofv3 kernel-trace stats (two-stream and single-stream), FETCH_SIZE /
# WRITE_SIZE passes of the bench (roofline traffic, whole-step bytes), SQ / byte PMC groups on enc2_block1,
# enc3_block1 and enc3_block2 at batch 32, and the other BASELINE configs at their per-GPU shape
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r6fin}
PART=${2:-AB}
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
[[ $PART == *A* ]] && run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $PART == *A* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $PART == *A* ]] && run bench 900 python bench.py
[[ $PART == *A* ]] && run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
export UNET_OVERLAP=0
[[ $PART == *A* ]] && run prof1s 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_1s -- $B
unset UNET_OVERLAP
[[ $PART == *A* ]] && run pmcF 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $B
[[ $PART == *A* ]] && run pmcW 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $B
export N=32
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
S="python tools/sep_one.py 1 128 128 64 128 10 x3"
[[ $PART == *B* ]] && run e2b1F 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e2b1_fetch -- $S
[[ $PART == *B* ]] && run e2b1W 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_e2b1_write -- $S
[[ $PART == *B* ]] && run e2b1S 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc -o ${TAG}_e2b1_sq -- $S
S="python tools/sep_one.py 1 64 64 128 256 10 x3"
[[ $PART == *B* ]] && run e3b1S 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b1_sq -- $S
export POOL=1
S="python tools/sep_one.py 1 64 64 256 256 10 x3"
[[ $PART == *B* ]] && run e3b2S 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc -o ${TAG}_e3b2_sq -- $S
unset POOL N
[[ $PART == *B* ]] && run cfg3 300 python bench.py --size 512 --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
[[ $PART == *B* ]] && run cfg4_b8 300 python bench.py --num-classes 21 --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
[[ $PART == *B* ]] && run cfg4_b32 300 python bench.py --num-classes 21 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
[[ $PART == *B* ]] && run cfg0 300 python bench.py --size 128 --batch 2 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --encoder-batch 0
[[ $PART == *B* ]] && run syncbn2 300 env UNET_DP_ONE_DEVICE=1 python bench.py --gpus 2 --sync-bn --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0
[[ $PART == *C* ]] && run bench_pinned 900 python bench.py
if [[ $PART == *S* ]]; then
  run sx_tests 600 python -u -m pytest tests/test_ops_gpu.py -k sepconv_bwd_fused -x -q --timeout 300 --timeout-method thread
  for i in 1 2 3; do
    run ab_sx1_$i 300 python bench.py --no-cpu-baseline --no-roofline --encoder-batch 0
    run ab_sx0_$i 300 python bench.py --no-cpu-baseline --no-roofline --encoder-batch 0 --no-x6-fused-bwd
  done
  run sx_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r6sx -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0
fi
if [[ $PART == *G* ]]; then
  run g_tests 600 python -u -m pytest tests/test_graph_predict_gpu.py -x -v --timeout 300 --timeout-method thread
  run g_predict 300 python tools/bench_predict.py 1 2 4 16 32
fi
exit 0
