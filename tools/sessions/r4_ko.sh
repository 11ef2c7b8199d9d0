#!/bin/bash
# round 4: X6 sepconv knock-outs at batch 32 + a bench line at HEAD
source "$(dirname "$0")/gpu_session.sh"
run ko 300 tools/lab/x6_ko_lab 32
run bench 300 python bench.py --no-cpu-baseline
