#!/bin/bash
# round 4: after stamps became the only step mark -- the A/B cells again, then the -m gpu suite
set -o pipefail
O=gpurun_out/r04_stamp_after
mkdir -p $O
timeout -k 10 300 python3 -u profiles/stamp_marks_ab.py > $O/after.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 600 bash profiles/configs_1gpu.sh > $O/configs_1gpu.log 2>&1
