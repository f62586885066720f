#!/bin/bash
# round 4: marks only on the steps a Timer reads -- the new GPU test, the A/B, then the -m gpu suite
set -o pipefail
O=gpurun_out/r04_marks
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_marks.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/marks_test.log 2>&1 &&
timeout -k 10 300 python3 -u profiles/timed_steps_ab.py > $O/ab.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $O/smoke.txt 2>&1
