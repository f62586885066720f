#!/bin/bash
# Round 3, call C: piece-size A/B of small copy launches, the bench under rocprofv3 (+ PMC),
# the README configuration through the CLI per mode.
out=${1:-gpurun_out/r03c}; mkdir -p $out
bash profiles/min_wg_ab.sh $PWD/$out/min_wg || exit 1
bash profiles/r03c_gpu.sh $out || exit 1
