#!/bin/bash
# usage: tools/sessions/gpu_bench_only.sh TAG -- the default bench line alone (e.g. after a PMC summary it
# reads was committed)
source "$(dirname "$0")/gpu_session.sh"
run bench_${1:-b} 900 python bench.py
