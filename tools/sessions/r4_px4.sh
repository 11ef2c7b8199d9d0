#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run px_check 240 python tools/lab_px.py 32 both
export N=32 SCHED=0
S="python tools/sep_one.py 1 128 128 128 128 10 x3"
run pmcF_0 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o px_F_0 -- $S
