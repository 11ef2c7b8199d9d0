#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run t_model 600 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread -k "schedules or determinism"
