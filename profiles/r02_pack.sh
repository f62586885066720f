#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# Round 2: pack / unpack / local-gather launches of the 8-GPU configs[2] plans on one MI355X
# (virtual GPUs): kernel trace with the local gather on the side stream (default) and fused
# into the pack launch (XG_SPLIT_LOCAL=0), then PMC traffic per launch class (separate passes).
export TMPDIR=/tmp
o=$PWD/gpurun_out/r02_pack; mkdir -p $o
for mode in split fused; do
  if [ $mode = fused ]; then export XG_SPLIT_LOCAL=0; else unset XG_SPLIT_LOCAL; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt_$mode -o run --output-format csv -- python3 profiles/pack_virtual.py > $o/run_$mode.txt 2> $o/run_$mode.err || exit 1
  python3 profiles/pack_summary.py $(find $o/kt_$mode -name run_kernel_trace.csv) > $o/summary_$mode.txt || exit 1
  REPS=20 timeout -k 10 120 python3 profiles/pack_virtual.py > $o/time_$mode.txt 2>&1 || exit 1
done
unset XG_SPLIT_LOCAL
REPS=3 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- python3 profiles/pack_virtual.py > /dev/null 2>&1 || exit 1
REPS=3 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- python3 profiles/pack_virtual.py > /dev/null 2>&1 || exit 1
python3 profiles/pack_pmc.py $(find $o/fetch -name run_counter_collection.csv) $(find $o/write -name run_counter_collection.csv) > $o/pmc.txt || exit 1
echo done
