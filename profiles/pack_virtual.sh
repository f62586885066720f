#!/bin/bash
# pack / unpack kernels of the 8-GPU configs[2] plans on one MI355X under rocprofv3
export TMPDIR=/tmp
o=$PWD/gpurun_out/pack; mkdir -p $o
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 profiles/pack_virtual.py > $o/run.txt 2> $o/run.err || exit 1
python3 profiles/pack_summary.py $(find $o/kt -name run_kernel_trace.csv | head -1) > $o/summary.txt || exit 1
cp $(find $o/kt -name run_kernel_stats.csv | head -1) $o/kernel_stats.csv
cat $o/run.txt $o/summary.txt
