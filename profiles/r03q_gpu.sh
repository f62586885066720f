#!/bin/bash
# Round 3, call Q: a split step's local part forking after its pack launch (XG_SPLIT_AFTER_PACK):
# GPU tests of the cross-GPU step forms (both orders), then GPU 0's configs[2] share alone, device
# time per run, 0 vs 1 interleaved 3 times.
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03q; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_virtual.py -m gpu -q -k "step_forms or one_gpu_share" --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for r in 1 2 3; do
  for a in 0 1; do
    XG_SPLIT_AFTER_PACK=$a timeout -k 10 120 python3 -u profiles/share_runtime.py >> $o/share_runtime.txt 2>&1 || { tail $o/share_runtime.txt; exit 1; }
  done
done
cat $o/share_runtime.txt
