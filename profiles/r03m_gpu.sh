#!/bin/bash
# Round 3, call M: the one-GPU-share hook's GPU test, then configs[4] at its stated size as GPU
# 0's share of the 8-GPU job (profiles/configs4_share.py).
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03m; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_virtual.py -m gpu -q -k "one_gpu_share or wave_copy" --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 600 python3 -u profiles/configs4_share.py > $o/configs4_share.txt 2>&1 || { tail -30 $o/configs4_share.txt; exit 1; }
cat $o/configs4_share.txt
