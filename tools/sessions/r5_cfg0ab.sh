# configs[0] shape (128x128, batch 2; host / launch-latency bound): HEAD b1b74cf vs this tree
set -e
B="--size 128 --batch 2 --steps 40 --warmup 10 --no-cpu-baseline --no-roofline --encoder-batch 0"
for i in 1 2 3; do
  timeout -k 10 300 python tools/abhead/bench.py $B > gpurun_out/c0_head_$i.log 2>&1
  timeout -k 10 300 python bench.py $B > gpurun_out/c0_new_$i.log 2>&1
done
