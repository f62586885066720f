#!/bin/bash
# round 4, call D: tests/test_gpu_baseline.py in suite order, output uncaptured (-s), RCCL
# warnings on, the watchdog at 60 s (writes gpurun_out/watchdog.txt if a test hangs)
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
NCCL_DEBUG=WARN XG_TEST_WATCHDOG=60 XG_WATCHDOG_LOG=$O/watchdog.txt timeout -k 10 400 python -u -m pytest \
    tests/test_gpu_baseline.py -x -v -s --timeout 600 --timeout-method thread > $O/gpu_baseline.log 2>&1
