#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# Round 3, call N: the product's cross-GPU copy launches as one real GPU runs them -- GPU 0's share
# of the configs[2] 8-GPU plans alone (profiles/share_launches.py), rocprofv3 kernel traces reduced
# per launch class, the wave copy on / off, two-sided and one-sided.
export TMPDIR=/tmp
o=$PWD/gpurun_out/r03n; mkdir -p $o
for rep in 1 2; do
for w in 1 0; do
  for f in 0 1; do
    ( export XG_COPY_WAVE=$w FORM=$f; timeout -k 10 120 rocprofv3 --kernel-trace -d $o/kt -o run --output-format csv -- \
      python3 profiles/share_launches.py > $o/share_w${w}_f${f}.txt 2>&1 ) || { tail -20 $o/share_w${w}_f${f}.txt; exit 1; }
    echo "== rep $rep XG_COPY_WAVE=$w FORM=$f" >> $o/summary.txt
    grep "^m" $o/share_w${w}_f${f}.txt >> $o/summary.txt
    python3 profiles/kernel_classes.py $(find $o/kt -name run_kernel_trace.csv) >> $o/summary.txt || exit 1
    rm -rf $o/kt
  done
done
done
cat $o/summary.txt
