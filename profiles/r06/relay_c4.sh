#!/bin/bash
# round 6: configs[4]'s relayed plans on the device before the driver's N = 8 run does it --
# the virtual 8-GPU job (copies every -c, RCCL at -c 1 / 8) and real 8-rank jobs (socket transport)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_baseline.py::test_config4_d8m_virtual8" \
  "tests/test_gpu_multirank.py::test_relay_form_config4_as_eight_rank_job" \
  --durations=8 > gpurun_out/r06/relay_c4.log 2>&1
