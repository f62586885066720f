#!/bin/bash
# round 6: the new relay-form GPU tests (every method, every step form), then the driver's N = 8
# command form with every rank on this GPU (profiles/r06/torchrun8.sh) at the round-6 budgets.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_virtual.py -k "relay_forms" --durations=8 > gpurun_out/r06/relay_forms_tests.log 2>&1 \
  || { echo "relay form tests rc=$?"; tail -30 gpurun_out/r06/relay_forms_tests.log; exit 1; }
tail -14 gpurun_out/r06/relay_forms_tests.log
bash profiles/r06/torchrun8.sh
