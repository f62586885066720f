#!/bin/bash
# round 4, call B: the whole -m gpu suite, smoke, and the default bench line at HEAD
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=25 \
    > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as G; G.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
