#!/bin/bash
# usage: tools/sessions/r6_pin.sh -- round 6: the default bench line once the PMC traffic summary pinned to this library
# build is committed (profiles/r6fin_traffic_*.json), so its roofline object carries the measured traffic
source "$(dirname "$0")/gpu_session.sh"
run bench_pinned 900 python bench.py
