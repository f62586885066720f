#!/bin/bash
# round 4, last: the two-ranks-one-GPU probe (expected to be refused by RCCL: its line), then the
# driver's three commands
set -o pipefail
O=gpurun_out/r04_final3
mkdir -p $O
bash profiles/r04_two_ranks_one_gpu.sh
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
