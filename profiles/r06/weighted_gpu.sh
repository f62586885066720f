#!/bin/bash
# round 6: the coalesced form's weighted two-hop split (configs[4] m7) on the device -- the virtual
# 8-GPU RCCL job's cost beside direct, and the GPU tests that now run it (configs[4] -d 8 MiB
# virtual 8-GPU, real 8-rank jobs, every method / step form).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
SPLIT=0 CASES=m7 timeout -k 10 300 python3 -u profiles/r06/relay_cost.py > gpurun_out/r06/relay_cost_m7.log 2>&1 || { echo "relay_cost rc=$?"; tail -5 gpurun_out/r06/relay_cost_m7.log; exit 1; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_baseline.py tests/test_gpu_multirank.py tests/test_gpu_virtual.py \
  -k "config4_d8m_virtual8 or relay" --durations=12 > gpurun_out/r06/weighted_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r06/weighted_tests.log; cat gpurun_out/r06/relay_cost_m7.log | grep virtual8; exit $rc
