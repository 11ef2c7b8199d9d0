#!/bin/bash
source "$(dirname "$0")/gpu_session.sh"
run split 300 python tools/lab_split_batch.py
