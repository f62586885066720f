#!/bin/bash
# round 6: the coalesced relay form (XG_RELAY_COALESCED) on the device -- (a) relay_cost.py's virtual
# 8-GPU RCCL job at configs[3] m9 / m10 in the direct, relay and coalesced forms; (b) the configs[3]
# full-size and configs[4] -d 8 MiB virtual 8-GPU tests and the real multi-rank relay tests, which
# now run both relay forms.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
SPLIT=0 timeout -k 10 300 python3 -u profiles/r06/relay_cost.py > gpurun_out/r06/relay_cost_coalesced.log 2>&1 || { echo "relay_cost rc=$?"; tail -5 gpurun_out/r06/relay_cost_coalesced.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_baseline.py tests/test_gpu_multirank.py -k "config3_full_size_virtual8 or config4_d8m_virtual8 or relay" \
  --durations=12 > gpurun_out/r06/coalesced_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r06/coalesced_tests.log; exit $rc
