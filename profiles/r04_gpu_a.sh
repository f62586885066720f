#!/bin/bash
# round 4, call A: the BASELINE-shape parity tests (tests/test_gpu_baseline.py) with per-test durations
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 900 python -u -m pytest tests/test_gpu_baseline.py -x -v --timeout 600 --timeout-method thread \
    --durations=0 > gpurun_out/r04a/gpu_baseline.log 2>&1
