#!/bin/bash
# Round 5: the real multi-rank tests (tests/test_gpu_multirank.py) and the relay form's virtual
# 8-GPU test at configs[3]'s full size on the one-GPU box, then an 8-rank bench.py rehearsal of
# the driver's N = 8 line (every rank on this GPU, XG_SHARE_GPU=1).
set -o pipefail
out=gpurun_out/r05_multirank
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py "tests/test_gpu_baseline.py::test_config3_full_size_virtual8" -x -v --timeout 300 --timeout-method thread --durations=0 > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -32 $out/tests.log; [ $rc -eq 0 ] || exit $rc
XG_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 5 --warmup 2 --baseline-budget 60 --cpu-configs-budget 60 > $out/bench8.json 2> $out/bench8.err
rc=$?; echo "bench8 rc=$rc"; tail -c 1500 $out/bench8.json; exit $rc
