#!/bin/bash
# same-box step A/B of the product library against tools/lab/$1 (an alternative build), ABAB
source "$(dirname "$0")/gpu_session.sh"
ALT=tools/lab/${1:?alt lib}
run a1 300 python bench.py --no-cpu-baseline
run b1 300 env UNET_HIP_LIB=$ALT python bench.py --no-cpu-baseline
run a2 300 python bench.py --no-cpu-baseline --encoder-batch 0
run b2 300 env UNET_HIP_LIB=$ALT python bench.py --no-cpu-baseline --encoder-batch 0
