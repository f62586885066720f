#!/bin/bash
# round 4, call C: the P256 virtual 8-GPU RCCL baseline cases alone, RCCL warnings on, a stack
# dump if one hangs (pytest-timeout 100 s, thread method)
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
NCCL_DEBUG=WARN timeout -k 10 170 python -u -m pytest tests/test_gpu_baseline.py -k "virtual8_rccl and cfg4" -x -v \
    --timeout 100 --timeout-method thread --durations=0 > $O/rccl_cfg4.log 2>&1
