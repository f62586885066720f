#!/bin/bash
# round 4, final: the driver's own forms -- `pytest tests/ -x -q -m gpu`, smoke(), `python bench.py`
set -o pipefail
O=gpurun_out/${OUT:-r04_final}
mkdir -p $O
timeout -k 10 1000 python -m pytest tests/ -x -q -m gpu > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
