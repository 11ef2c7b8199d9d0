# kernel trace of configs[4] at batch 8 (21 classes) for the step-trace breakdown
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4t -o c4b8 -- python bench.py --num-classes 21 --batch 8 --steps 8 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0 > gpurun_out/c4t.log 2>&1
