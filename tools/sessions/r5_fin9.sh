# kernel traces: HEAD vs this tree (bn_finalize / bn_bwd_stats loads batched)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="--steps 8 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fin9 -o head -- python tools/abhead/bench.py $B > gpurun_out/fin9_head.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fin9 -o new -- python bench.py $B > gpurun_out/fin9_new.log 2>&1
