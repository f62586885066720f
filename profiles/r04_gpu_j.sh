#!/bin/bash
# round 4, call J: BASELINE configs through the drop-in CLI on one MI355X beside the reference
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 900 bash profiles/configs_1gpu.sh > $O/configs_1gpu.txt 2>&1
