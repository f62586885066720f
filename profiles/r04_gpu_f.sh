#!/bin/bash
# round 4, call F: the CLI at the BASELINE shapes against the reference's masked reports
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -k baseline_shapes -x -v --timeout 600 --timeout-method thread \
    --durations=0 > $O/cli_baseline.log 2>&1
