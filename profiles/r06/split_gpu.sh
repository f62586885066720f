#!/bin/bash
# round 6: the coalesced form's large-piece split (rc_split) and the relay-form GPU tests at the
# last code
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_virtual.py tests/test_gpu_baseline.py tests/test_gpu_multirank.py \
  -k "relay or config4_d8m_virtual8 or config3_full_size" --durations=12 > gpurun_out/r06/split_tests.log 2>&1
rc=$?; tail -22 gpurun_out/r06/split_tests.log; exit $rc
