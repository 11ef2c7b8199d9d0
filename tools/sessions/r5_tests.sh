set -e
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r5t_tests.log 2>&1
