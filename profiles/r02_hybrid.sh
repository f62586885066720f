#!/bin/bash
# engine segments in the virtual 8-GPU README-config plans, engine on / off, rocprofv3 kernel traces
export TMPDIR=/tmp
o=$PWD/gpurun_out/r02_hybrid; mkdir -p $o
for mode in engine eager; do
  if [ $mode = eager ]; then export XG_ENGINE_MAX_STEP=0; else unset XG_ENGINE_MAX_STEP; fi
  REPS=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt_$mode -o run --output-format csv -- python3 profiles/hybrid_virtual.py > $o/run_$mode.txt 2> $o/run_$mode.err || exit 1
  cp $(find $o/kt_$mode -name run_kernel_stats.csv) $o/stats_$mode.csv
done
echo done
