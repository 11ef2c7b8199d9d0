# kernel traces of the step with the in-launch BN finish on / off
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-roofline --encoder-batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fin3 -o on -- $B > gpurun_out/fin3_on.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fin3 -o off -- $B --no-fin-in-launch > gpurun_out/fin3_off.log 2>&1
