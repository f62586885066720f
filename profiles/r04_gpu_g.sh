#!/bin/bash
# round 4, call G: the widened random sweep -- 600 one-GPU + 300 virtual 2/3/4/8-GPU + 120 virtual
# P = 48..256 configurations, every method, against the oracle's closed form
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
XG_RANDOM_N1=600 XG_RANDOM_NV=300 XG_RANDOM_NL=120 timeout -k 10 1000 python -u -m pytest tests/test_gpu_random.py -x -q \
    --timeout 600 --timeout-method thread -p no:cacheprovider > $O/random_sweep.log 2>&1
