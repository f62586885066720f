#!/bin/bash
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
# Piece size per launch (XG_COPY_BALANCE): the configs[2] 8-GPU pack / unpack / gather classes
# on one MI355X (virtual GPUs) and the bench line, with the balanced rule (1) and with 32 KiB
# pieces everywhere (0); rocprofv3 kernel traces, per class.
export TMPDIR=/tmp
o=${1:-$PWD/gpurun_out/balance_ab}; mkdir -p $o
for b in 0 1 0 1; do
  XG_COPY_BALANCE=$b timeout -k 10 120 rocprofv3 --kernel-trace -d $o/kt_$b -o run --output-format csv -- python3 profiles/pack_virtual.py > /dev/null 2>> $o/err.txt || exit 1
  echo "# XG_COPY_BALANCE=$b" >> $o/summary.txt
  python3 profiles/pack_summary.py $(find $o/kt_$b -name run_kernel_trace.csv) 256=4194304,1792=29360128 >> $o/summary.txt || exit 1
  rm -rf $o/kt_$b
done
for b in 0 1; do
  XG_COPY_BALANCE=$b timeout -k 10 300 python3 bench.py --no-cpu-baseline > $o/bench_$b.json 2>> $o/err.txt || exit 1
  python3 -c "import json,sys; d=json.load(open('$o/bench_$b.json')); print('bench balance=$b', d['value'], d['roofline']['avg_launch_us'])" >> $o/summary.txt
done
cat $o/summary.txt
