#!/bin/bash
# Round 5: multi-rank tests + relay virtual test, then the N = 8 torchrun rehearsal.
set -o pipefail
out=gpurun_out/r05_check
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py "tests/test_gpu_baseline.py::test_config3_full_size_virtual8" -x -v --timeout 300 --timeout-method thread --durations=8 > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -14 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r05/torchrun8.sh
