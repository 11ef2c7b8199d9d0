# the bench line with the committed PMC traffic pinned to this library, then the other configs
set -e
timeout -k 10 600 python bench.py > gpurun_out/pinned.log 2>&1
bash tools/sessions/gpu_cfgs.sh
