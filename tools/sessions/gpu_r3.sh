#!/bin/bash
# usage: tools/sessions/gpu_r2.sh TAG [steps...] -- round-3 GPU session: steps from {parity,tests,smoke,bench,prof,prof1s,pmc}
source "$(dirname "$0")/gpu_session.sh"
TAG=${1:-r3}; shift
export UNET_PARITY_LOG=gpurun_out/parity_${TAG}.jsonl
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --encoder-batch 0"
for s in "$@"; do
  case $s in
    parity) run parity 600 python -u -m pytest tests/test_parity_sizes_gpu.py -x -v --timeout 300 --timeout-method thread ;;
    tests) run tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run benchq 300 python bench.py --no-cpu-baseline ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG} -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder-batch 0 ;;
    prof1s) UNET_OVERLAP=0 run prof1s 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ${TAG}_1s -- $B ;;
    pmc) run pmcF 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- $B
         run pmcW 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- $B ;;
  esac
done
